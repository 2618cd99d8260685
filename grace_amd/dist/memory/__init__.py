"""Import-path compatibility with grace_dl.dist.memory (re-exports)."""
