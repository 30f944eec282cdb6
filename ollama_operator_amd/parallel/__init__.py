"""Parallelism: tensor-parallel serving over RCCL/xGMI (`tp`). Data parallelism is one server pod
per GPU (operator `spec.replicas`); the Megatron sharding plan itself lives with the weights
(engine/weights.py) and the collectives in engine/runner.py."""
from .tp import TPControl, TPRunnerProxy, load_tp_runner, start_leader, tp_size_from_env

__all__ = ["TPControl", "TPRunnerProxy", "load_tp_runner", "start_leader", "tp_size_from_env"]
