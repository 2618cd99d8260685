"""Import-path compatibility with grace_dl.torch.compressor (re-exports)."""
