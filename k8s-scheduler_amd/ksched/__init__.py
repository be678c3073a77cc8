"""ksched -- MI355X-native scheduling core with the semantics of yinwoods/k8s-scheduler's anchor package.

Product surface:
  ksched.Engine            C-ABI engine (libksched.so): exact and batched modes, one GPU / node shard
  ksched.host.FakeCluster  predicate / priorities / schedulePod / schedulePods mirror (in-memory apiserver)
  ksched.dist              node-sharded multi-GPU helpers (RCCL inside the engine)
  ksched.cluster           seeded synthetic clusters for the BASELINE configs
"""
from ._lib import (DOMAIN_ALL, DOMAIN_FEASIBLE, MODE_AUTO, MODE_BATCHED, MODE_EXACT, NO_FIT, NO_POSITIVE_SCORE,
                   PRIORITY_BEST_PRICE, PRIORITY_RESOURCE, KschedError, lib)
from .engine import Engine, Group, engine_for

__all__ = ["Engine", "Group", "engine_for", "KschedError", "lib", "MODE_AUTO", "MODE_BATCHED", "MODE_EXACT",
           "PRIORITY_RESOURCE", "PRIORITY_BEST_PRICE", "DOMAIN_ALL", "DOMAIN_FEASIBLE", "NO_FIT",
           "NO_POSITIVE_SCORE"]
