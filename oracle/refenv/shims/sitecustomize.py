"""Environment glue so the reference imports under astropy 4.3.1 + numpy 1.26 in this
container (oracle harness only; never shipped to, or run on, the GPU box)."""
import numpy as _np

for _n, _v in {"asscalar": lambda a: a.item(), "alen": lambda a: len(a), "float": float, "int": int,
               "bool": bool, "object": object, "complex": complex, "str": str, "long": int,
               "unicode": str}.items():
    if not hasattr(_np, _n):
        setattr(_np, _n, _v)

import importlib.abc as _abc
import importlib.machinery as _mach
import sys as _sys

_TARGET = "astropy.units.quantity_helper.function_helpers"


def _patch(mod):
    def concatenate(arrays, axis=0, out=None, dtype=None, casting="same_kind"):
        arrays, kwargs, unit, out = mod._iterable_helper(*arrays, out=out, axis=axis)
        if dtype is not None:
            kwargs["dtype"] = dtype
        kwargs["casting"] = casting
        return (arrays,), kwargs, unit, out

    mod.FUNCTION_HELPERS[_np.concatenate] = concatenate


class _Loader(_abc.Loader):
    def __init__(self, inner):
        self.inner = inner

    def create_module(self, spec):
        return self.inner.create_module(spec)

    def exec_module(self, module):
        self.inner.exec_module(module)
        _patch(module)


class _Finder(_abc.MetaPathFinder):
    def find_spec(self, name, path, target=None):
        if name != _TARGET:
            return None
        spec = _mach.PathFinder.find_spec(name, path)
        if spec is not None:
            spec.loader = _Loader(spec.loader)
        return spec


_sys.meta_path.insert(0, _Finder())
