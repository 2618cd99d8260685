"""Import-path compatibility with grace_dl.dist.communicator (re-exports)."""
