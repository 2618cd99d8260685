"""Import-path compatibility with grace_dl.torch.memory (re-exports)."""
