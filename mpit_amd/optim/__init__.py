"""Distributed and local optimizers of mpiT (SURVEY §2.4, O1–O13)."""
from .distributed import downpour, eamsgd, easgd, msgd

__all__ = ["downpour", "eamsgd", "easgd", "msgd"]
