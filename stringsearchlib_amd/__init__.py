"""stringsearchlib_amd — MI355X-native n-gram fuzzy search (drop-in for StringSearchLib's DLL).

The product is libngram_search.so (C ABI in include/ngram_search.h); this package is a thin
host-side mirror of the reference interface over it. See DESIGN.md.
"""
from .index import INT32_MAX, StringIndex, WideStringIndex  # noqa: F401
from . import _native, synth  # noqa: F401

__all__ = ["StringIndex", "WideStringIndex", "INT32_MAX"]
