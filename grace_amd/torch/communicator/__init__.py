"""Import-path compatibility with grace_dl.torch.communicator (re-exports)."""
