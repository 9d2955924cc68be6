"""openwhisk_amd -- MI355X-native batched invoker scheduler for OpenWhisk's controller (ShardingContainerPoolBalancer
schedule() hot path).  C ABI: include/owgs.h; HIP engine: openwhisk_amd/csrc; host mirror: balancer.py."""
from ._lib import OwgsError, build, header_functions, lib  # noqa: F401
from .balancer import Action, GpuShardingContainerPoolBalancer, InvokerHealth  # noqa: F401

__all__ = ["GpuShardingContainerPoolBalancer", "InvokerHealth", "Action", "OwgsError", "build", "lib",
           "header_functions"]
