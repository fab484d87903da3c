"""Distributed and local optimizers of mpiT (SURVEY §2.4, O1–O13).

Torch-optim convention: ``w, [fx] = optim.NAME(opfunc, w, config, state)``."""
from .adaptive import (
    adadelta,
    adadeltasingle,
    adagrad,
    adagradsingle,
    adam,
    adamax,
    adamaxsingle,
    adamsingle,
    rmsprop,
    rmspropsingle,
)
from .distributed import downpour, eamsgd, easgd, msgd

ALL = {
    "msgd": msgd, "sgd": msgd, "downpour": downpour, "eamsgd": eamsgd, "easgd": easgd,
    "rmsprop": rmsprop, "adam": adam, "adamax": adamax, "adagrad": adagrad, "adadelta": adadelta,
    "rmspropsingle": rmspropsingle, "adamsingle": adamsingle, "adamaxsingle": adamaxsingle,
    "adagradsingle": adagradsingle, "adadeltasingle": adadeltasingle,
}

__all__ = sorted(ALL) + ["ALL"]
