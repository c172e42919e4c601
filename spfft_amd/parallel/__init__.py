"""Communicators and distribution helpers.

``LocalGroup``       N in-process ranks (threads); GPU data plane = peer copies.
``TorchDistComm``    control plane over torch.distributed (gloo group); the GPU
                     data plane is RCCL, bootstrapped through it.
"""
from .comm import Communicator, LocalGroup, TorchDistComm, run_ranks  # noqa: F401
from .distributed import DistributedSetup, even_planes, make_distributed  # noqa: F401
