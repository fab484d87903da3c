"""Parallelism: parameter server (async DP, EASGD, sharding, SSP) and synchronous DP."""
from .ps import PClient, PServer, ServerOpt, pClient, pServer, shard_ranges

__all__ = ["PClient", "PServer", "ServerOpt", "pClient", "pServer", "shard_ranges"]
