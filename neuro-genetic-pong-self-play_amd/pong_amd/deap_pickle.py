"""Reference checkpoint pickles (utils.save_checkpoint, utils.py:116-125) in
both directions, with or without DEAP installed.

A checkpoint the reference writes pickles DEAP's classes by their module
paths: ``deap.creator.Individual`` / ``deap.creator.Fitness`` (classes that
``creator.create`` makes inside ``deap.creator``, ga.py:80-81),
``deap.tools.support.HallOfFame`` (ga.py:78) and ``_operator.eq`` (the hall
of fame's ``similar``).  DEAP is not installable offline, so the drop-in
``ga`` falls back to the in-repo restatement (``pong_amd.deap_compat``), whose
classes live at other paths.  This module bridges the two:

* ``load`` unpickles with a ``find_class`` that resolves ``deap.*`` to the
  restatement when deap is absent (and the restatement's own paths, written by
  older builds, to real DEAP when it is present).  It resolves only the
  globals a checkpoint can contain (the DEAP classes above, ``copyreg`` /
  ``operator.eq``, numpy scalars and arrays), each by its exact
  ``(module, name)`` pair; anything else -- any other name of an allowed
  module, or a dotted name -- raises ``pickle.UnpicklingError`` instead of
  importing it.
* ``dump`` pickles restatement objects under DEAP's module paths, so the
  reference's ``ga.load_population_from_file`` (ga.py:41-53, real DEAP)
  reads the build's exports.  The C pickler resolves a class by importing its
  ``__module__``, so for the duration of the dump the restatement classes take
  DEAP's ``__module__`` and stand-in ``deap`` modules exposing them are placed
  in ``sys.modules`` (only when real DEAP is absent; restored afterwards,
  under a lock).
"""
from __future__ import annotations

import contextlib
import importlib
import pickle
import sys
import threading
import types

_LOCK = threading.Lock()

# DEAP's module path of every class a checkpoint can hold -> the restatement's
# (module, name).  Real DEAP defines HallOfFame/Statistics/Logbook in
# deap/tools/support.py and re-exports them from deap.tools.
_DEAP_TO_COMPAT = {
    ("deap.creator", "Individual"): ("pong_amd.deap_compat.creator", "Individual"),
    ("deap.creator", "Fitness"): ("pong_amd.deap_compat.creator", "Fitness"),
    ("deap.base", "Fitness"): ("pong_amd.deap_compat.base", "Fitness"),
    ("deap.base", "Toolbox"): ("pong_amd.deap_compat.base", "Toolbox"),
    ("deap.tools.support", "HallOfFame"): ("pong_amd.deap_compat.tools", "HallOfFame"),
    ("deap.tools.support", "Statistics"): ("pong_amd.deap_compat.tools", "Statistics"),
    ("deap.tools.support", "Logbook"): ("pong_amd.deap_compat.tools", "Logbook"),
    ("deap.tools", "HallOfFame"): ("pong_amd.deap_compat.tools", "HallOfFame"),
    ("deap.tools", "Statistics"): ("pong_amd.deap_compat.tools", "Statistics"),
    ("deap.tools", "Logbook"): ("pong_amd.deap_compat.tools", "Logbook"),
}
_COMPAT_TO_DEAP = {}
for _d, _c in _DEAP_TO_COMPAT.items():
    if _d[0] != "deap.tools":  # support.* is the defining module
        _COMPAT_TO_DEAP.setdefault(_c, _d)

# other globals a save_checkpoint pickle may name
_ALLOWED = {
    ("copyreg", "_reconstructor"), ("copy_reg", "_reconstructor"),
    ("builtins", "object"), ("builtins", "list"), ("builtins", "tuple"), ("builtins", "dict"),
    ("builtins", "set"), ("builtins", "frozenset"), ("builtins", "float"), ("builtins", "int"),
    ("__builtin__", "object"), ("__builtin__", "list"),
    ("numpy", "dtype"), ("numpy", "ndarray"),
    ("numpy.core.multiarray", "scalar"), ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "scalar"), ("numpy._core.multiarray", "_reconstruct"),
    # HallOfFame.similar (operator.eq, ga.py:78): the only operator global a
    # checkpoint holds.  Exact pairs, never whole modules: _operator's
    # attrgetter / getitem / methodcaller reach eval through a reconstructor's
    # __globals__ with GLOBAL and REDUCE alone.
    ("_operator", "eq"), ("operator", "eq"),
}


def deap_installed() -> bool:
    try:
        importlib.import_module("deap.creator")
        return True
    except ImportError:
        return False


def _ensure_creator_classes(creator_mod):
    """ga.py:80-81's classes: ``creator.create`` runs at ga import; a loader
    used before that (e.g. checkpoint.read_reference) creates them itself."""
    if not hasattr(creator_mod, "Fitness") or not hasattr(creator_mod, "Individual"):
        base = importlib.import_module(creator_mod.__name__.rsplit(".", 1)[0] + ".base")
        if not hasattr(creator_mod, "Fitness"):
            creator_mod.create("Fitness", base.Fitness, weights=(1.0,))
        if not hasattr(creator_mod, "Individual"):
            creator_mod.create("Individual", list, fitness=creator_mod.Fitness)


class CheckpointUnpickler(pickle.Unpickler):
    """``pickle.Unpickler`` for save_checkpoint files (see module docstring)."""

    def __init__(self, fh, use_deap: bool | None = None):
        super().__init__(fh)
        self.use_deap = deap_installed() if use_deap is None else use_deap

    def find_class(self, module, name):
        key = (module, name)
        if "." in name:  # protocol 4 resolves dotted names attribute by attribute
            raise pickle.UnpicklingError(f"checkpoint names {module}.{name}: dotted names are refused")
        if key in _DEAP_TO_COMPAT or key in _COMPAT_TO_DEAP:
            if self.use_deap:
                module, name = _COMPAT_TO_DEAP.get(key, key)
            else:
                module, name = _DEAP_TO_COMPAT.get(key, key)
            mod = importlib.import_module(module)
            if module.endswith("creator"):
                _ensure_creator_classes(mod)
            return getattr(mod, name)
        if key in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"checkpoint names {module}.{name}, which a save_checkpoint "
                                     "file never holds; refusing to import it")


def load(fh, use_deap: bool | None = None):
    """``pickle.load`` of a save_checkpoint file (ga.py:44-45)."""
    return CheckpointUnpickler(fh, use_deap=use_deap).load()


def loads(data: bytes, use_deap: bool | None = None):
    import io
    return load(io.BytesIO(data), use_deap=use_deap)


@contextlib.contextmanager
def _deap_paths():
    """Restatement classes pickle as DEAP's while the context is open."""
    from .deap_compat import creator as c_creator
    _ensure_creator_classes(c_creator)
    with _LOCK:
        saved_mods = {}
        saved_attrs = []
        made = {}
        try:
            for (cmod, cname), (dmod, dname) in _COMPAT_TO_DEAP.items():
                cls = getattr(importlib.import_module(cmod), cname, None)
                if cls is None:
                    continue
                for part in ("deap", "deap.tools", dmod):
                    if part not in made:
                        saved_mods[part] = sys.modules.get(part)
                        made[part] = types.ModuleType(part)
                        sys.modules[part] = made[part]
                setattr(made[dmod], dname, cls)
                saved_attrs.append((cls, cls.__module__, cls.__qualname__))
                cls.__module__, cls.__qualname__ = dmod, dname
            yield
        finally:
            for cls, mod, qual in saved_attrs:
                cls.__module__, cls.__qualname__ = mod, qual
            for part, old in saved_mods.items():
                if old is None:
                    sys.modules.pop(part, None)
                else:
                    sys.modules[part] = old


def dump(obj, fh, protocol: int | None = None) -> None:
    """``pickle.dump`` (utils.py:124-125) naming DEAP's classes by DEAP's paths."""
    if deap_installed():
        pickle.dump(obj, fh, protocol=protocol)
        return
    with _deap_paths():
        pickle.dump(obj, fh, protocol=protocol)


def global_names(data: bytes) -> set:
    """Every ``module.name`` global a pickle refers to (for tests / inspection)."""
    import pickletools
    out, pushed, memo = set(), [], {}
    for op, arg, _ in pickletools.genops(data):
        if op.name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE", "BINUNICODE8"):
            pushed.append(arg)
        elif op.name in ("BINGET", "LONG_BINGET", "GET"):
            pushed.append(memo.get(arg))
        elif op.name == "MEMOIZE":
            memo[len(memo)] = pushed[-1] if pushed else None
            continue
        elif op.name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = pushed[-1] if pushed else None
            continue
        elif op.name == "STACK_GLOBAL":
            out.add(f"{pushed[-2]}.{pushed[-1]}")
            pushed.append(None)
        elif op.name in ("GLOBAL", "INST"):
            out.add(arg.replace(" ", "."))
            pushed.append(None)
        else:
            pushed.append(None)
    return out
