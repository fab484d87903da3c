"""Utilities: flat parameter storage, serialisation, timing, checkpointing, logging."""
from .flat import FlatParams
from .serialize import deserialize, serialize

__all__ = ["FlatParams", "serialize", "deserialize"]
