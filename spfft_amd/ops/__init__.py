"""Native-library bindings (ctypes) and low-level helpers."""
from ._lib import lib, library_path  # noqa: F401
