"""Checkpoints of the device GA (pong_amd.evolve.DeviceGA).

Two formats:

* the build's tensor checkpoint -- a safetensors file (8-byte little-endian
  header length, JSON header, raw little-endian tensor bytes), written block
  by block from the device so a 70 GB wide-MLP population never sits in host
  memory whole; ``safetensors.safe_open`` reads it (lazily) like any other.
  Tensors: ``population`` [P, G], ``fitness`` [P] f64, ``valid`` [P] u8,
  ``hall_of_fame`` [hof_n, G] (best first), ``hof_fitness`` [hof_n] f64.
  Metadata: the DeviceGA configuration, generation and logbook (JSON).
* the reference's pickle (save_checkpoint, utils.py:116-125):
  ``{population: [Individual], hall_of_fame: HallOfFame, rndstate:
  random.getstate(), network_shape}``, which ga.load_population_from_file
  (ga.py:41-53) resumes from; ``export_reference`` / ``import_reference``
  convert between the two.  Classes are pickled and resolved by DEAP's module
  paths in both directions (``deap_pickle``), so the reference reads the
  build's exports and the build reads the reference's checkpoints whether or
  not deap is installed.
"""
from __future__ import annotations

import datetime
import json
import os
import random
import struct

import numpy as np
import torch

from . import deap_pickle

FORMAT = "pong_amd.device_ga/1"
_DT = {torch.float64: "F64", torch.float32: "F32", torch.int64: "I64", torch.int32: "I32", torch.uint8: "U8"}
_TD = {v: k for k, v in _DT.items()}
_CONFIG_KEYS = ("nodes", "population_size", "hof_size", "tournsize", "bias", "dtype", "n_games", "schedule",
                "cxpb", "mutpb", "alpha", "mu", "sigma", "indpb", "seed", "physics_seed", "precision", "kernel",
                "hof_block_rows")


def write_tensors(path: str, tensors: dict, metadata: dict, block_bytes: int = 1 << 28) -> None:
    """Write a safetensors file from (possibly device) tensors, block by block."""
    header, off = {}, 0
    for name, t in tensors.items():
        nbytes = t.numel() * t.element_size()
        header[name] = {"dtype": _DT[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + nbytes]}
        off += nbytes
    header["__metadata__"] = {str(k): str(v) for k, v in metadata.items()}
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    tmp = path + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(struct.pack("<Q", len(hb)))
        fh.write(hb)
        for t in tensors.values():
            flat = t.detach().contiguous().reshape(-1)
            step = max(1, block_bytes // max(t.element_size(), 1))
            for i in range(0, flat.numel(), step):
                fh.write(flat[i:i + step].cpu().numpy().tobytes())
    os.replace(tmp, path)


def read_tensors(path: str, device=None, block_bytes: int = 1 << 28):
    """(tensors, metadata) of a safetensors file; tensors are copied to
    ``device`` block by block (host memory holds one block at a time)."""
    from safetensors import safe_open
    out = {}
    with safe_open(path, framework="pt", device="cpu") as f:
        meta = dict(f.metadata() or {})
        for name in f.keys():
            sl = f.get_slice(name)
            shape = list(sl.get_shape())
            dtype = _TD[sl.get_dtype()]
            t = torch.empty(shape, dtype=dtype, device=device or "cpu")
            if not shape or shape[0] == 0:
                if shape:
                    out[name] = t
                else:
                    out[name] = f.get_tensor(name).to(t.device)
                continue
            row_bytes = max(1, int(np.prod(shape[1:], dtype=np.int64)) * t.element_size())
            rows = max(1, block_bytes // row_bytes)
            for r0 in range(0, shape[0], rows):
                t[r0:r0 + rows] = sl[r0:r0 + rows].to(t.device)
            out[name] = t
    return out, meta


def _config(ga) -> dict:
    return {"nodes": ga.nodes, "population_size": ga.P, "hof_size": ga.H, "tournsize": ga.tournsize,
            "bias": ga.bias, "dtype": str(ga.dtype).replace("torch.", ""), "n_games": ga.n_games,
            "schedule": ga.schedule, "cxpb": ga.cxpb, "mutpb": ga.mutpb, "alpha": ga.alpha, "mu": ga.mu,
            "sigma": ga.sigma, "indpb": ga.indpb, "seed": ga.seed, "physics_seed": ga.physics_seed,
            "precision": ga.precision, "kernel": ga.kernel, "hof_block_rows": ga.hof_block_rows}


def save(ga, path: str) -> str:
    """Write the DeviceGA state (population, fitness, hall of fame, generation,
    logbook).  A sharded run (ga.shard_vary) holds only its shard's rows of
    the population: every rank calls save (one all-gather of the rows)."""
    tensors = {"population": ga.population_full(), "fitness": ga.fitness, "valid": ga.valid.to(torch.uint8),
               "hall_of_fame": ga.hall_of_fame,
               "hof_fitness": torch.from_numpy(np.ascontiguousarray(ga.hof_member_fitness))}
    meta = {"format": FORMAT, "config": json.dumps(_config(ga)), "generation": ga.generation,
            "logbook": json.dumps(ga.logbook)}
    write_tensors(path, tensors, meta)
    return path


def load(path: str, device=None, group=None):
    """A DeviceGA restored from ``save``: stepping it continues the saved run."""
    from .evolve import DeviceGA
    t, meta = read_tensors(path, device=device)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint (format={meta.get('format')!r})")
    cfg = json.loads(meta["config"])
    dtype = getattr(torch, cfg.pop("dtype"))
    nodes, P = cfg.pop("nodes"), cfg.pop("population_size")
    ga = DeviceGA(nodes, P, dtype=dtype, device=device, group=group, **cfg)
    ga.set_population(t["population"], t["fitness"], t["valid"])
    ga.set_hall_of_fame(t["hall_of_fame"], t["hof_fitness"].cpu().numpy())
    ga.generation = int(meta["generation"])
    ga.logbook = json.loads(meta["logbook"])
    return ga


# ------------------------------------------------------ reference pickle
def _deap():
    try:
        from deap import base, creator, tools
    except ImportError:
        from .deap_compat import base, creator, tools
    if not hasattr(creator, "Fitness"):
        creator.create("Fitness", base.Fitness, weights=(1.0,))
    if not hasattr(creator, "Individual"):
        creator.create("Individual", list, fitness=creator.Fitness)
    return creator, tools


def export_reference(state, path: str = None) -> str:
    """Write ``state`` (a DeviceGA, or any object with ``nodes``, ``H``,
    ``population``, ``fitness``, ``valid``, ``hall_of_fame`` and
    ``hof_member_fitness``) in save_checkpoint's pickle format (utils.py:116-125),
    to checkpoints/checkpoints/c_HH_MM_SS.pkl by default."""
    creator, tools = _deap()
    genes = state.population.double().cpu().numpy()
    fit = state.fitness.double().cpu().numpy()
    valid = state.valid.bool().cpu().numpy()
    population = []
    for r in range(genes.shape[0]):
        ind = creator.Individual(genes[r].tolist())
        if valid[r]:
            ind.fitness.values = (float(fit[r]),)
        population.append(ind)
    hof = tools.HallOfFame(int(state.H))
    hof_genes = state.hall_of_fame.double().cpu().numpy()
    for row, f in zip(hof_genes, state.hof_member_fitness):
        ind = creator.Individual(row.tolist())
        ind.fitness.values = (float(f),)
        hof.items.append(ind)                      # best first
    hof.keys = [ind.fitness for ind in reversed(hof.items)]  # ascending
    payload = {"population": population, "hall_of_fame": hof, "rndstate": random.getstate(),
               "network_shape": list(state.nodes)}
    if path is None:
        os.makedirs(os.path.join("checkpoints", "checkpoints"), exist_ok=True)
        stamp = datetime.datetime.now().strftime("%H_%M_%S")
        path = os.path.join("checkpoints", "checkpoints", f"c_{stamp}.pkl")
    with open(path, "wb") as fh:
        deap_pickle.dump(payload, fh)  # DEAP's class paths, readable by the reference's ga.py
    return path


def read_reference(path: str) -> dict:
    """Arrays of a save_checkpoint pickle written by this build or by a run of
    the reference on this machine (never a file shipped inside the reference):
    population genes/fitness/valid, hall-of-fame genes/fitness (best first),
    network_shape."""
    with open(path, "rb") as fh:
        cp = deap_pickle.load(fh)
    pop = cp["population"]
    genes = np.array([list(ind) for ind in pop], dtype=np.float64)
    valid = np.array([ind.fitness.valid for ind in pop], dtype=bool)
    fit = np.array([ind.fitness.values[0] if ind.fitness.valid else 0.0 for ind in pop], dtype=np.float64)
    hof = cp.get("hall_of_fame")
    items = list(hof.items) if hof is not None else []
    hof_genes = np.array([list(i) for i in items], dtype=np.float64).reshape(len(items), genes.shape[1] if len(pop) else 0)
    hof_fit = np.array([i.fitness.values[0] for i in items], dtype=np.float64)
    return {"genes": genes, "fitness": fit, "valid": valid, "hof_genes": hof_genes, "hof_fitness": hof_fit,
            "hof_size": hof.maxsize if hof is not None else None, "network_shape": cp.get("network_shape")}


def import_reference(path: str, device=None, **kw):
    """A DeviceGA holding a save_checkpoint pickle's population and hall of fame."""
    from .evolve import DeviceGA
    r = read_reference(path)
    nodes = kw.pop("nodes", r["network_shape"])
    if r["hof_size"] is not None:
        kw.setdefault("hof_size", r["hof_size"])
    ga = DeviceGA(nodes, r["genes"].shape[0], device=device, **kw)
    ga.set_population(torch.from_numpy(r["genes"]), torch.from_numpy(r["fitness"]), torch.from_numpy(r["valid"]))
    ga.set_hall_of_fame(torch.from_numpy(r["hof_genes"]), r["hof_fitness"])
    # generation -1: the first step is eaSimple's generation 0 -- evaluate the
    # invalid individuals only (none, for a reference checkpoint) and update the
    # hall of fame with the loaded population, as a resumed main() does
    return ga
