from ..helper import grace_from_params  # noqa: F401
