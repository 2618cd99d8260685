"""Import-path compatibility with grace_dl.dist.compressor (re-exports)."""
