"""grace_amd: MI355X-native gradient compression framework (GRACE capabilities)."""
__version__ = "0.1.0"
