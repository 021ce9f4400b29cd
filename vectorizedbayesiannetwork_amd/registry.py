"""Name -> class registries for the accelerated engines (mirrors reference core/registry.py:7-43).

Keys are the reference's own registry keys, so ``set_inference_method("importance_sampling")``
selects the HIP implementation here exactly as it selects the CPU one in the reference.
Duplicate registration raises ``ValueError`` like the reference decorators (registry.py:18-19).
"""
from __future__ import annotations

from typing import Callable, Dict, Type, TypeVar

T = TypeVar("T")

INFERENCE_REGISTRY: Dict[str, Type] = {}
SAMPLING_REGISTRY: Dict[str, Type] = {}


def _register(registry: Dict[str, Type], name: str) -> Callable[[Type[T]], Type[T]]:
    key = name.lower().strip()

    def deco(cls: Type[T]) -> Type[T]:
        if key in registry:
            raise ValueError(f"Duplicate registry key '{key}' for {cls.__name__}")
        registry[key] = cls
        return cls

    return deco


def register_inference(name: str):
    return _register(INFERENCE_REGISTRY, name)


def register_sampling(name: str):
    return _register(SAMPLING_REGISTRY, name)
