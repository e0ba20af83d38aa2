"""Per-process device state: one Evaluator per (shape, bias, dtype, precision),
created on first use on the configured device (config.DEVICE)."""
from __future__ import annotations

import threading

import numpy as np
import torch

from . import device as D

_lock = threading.Lock()
_evaluators = {}


def _torch_dtype(name: str):
    return {"float64": torch.float64, "float32": torch.float32}[name]


def evaluator(nodes, bias=True, n_games=6, genome_dtype="float64", precision="certified",
              seed=0, device="cuda", timeout_thresh=0, win_score=0) -> D.Evaluator:
    key = (tuple(int(n) for n in nodes), bool(bias), int(n_games), genome_dtype, precision, int(seed), str(device),
           int(timeout_thresh), int(win_score))
    with _lock:
        ev = _evaluators.get(key)
        if ev is None:
            dev = torch.device(device)
            if dev.type == "cuda" and dev.index is None:
                dev = torch.device("cuda", torch.cuda.current_device())
            ev = D.Evaluator(list(nodes), bias=bias, dtype=_torch_dtype(genome_dtype), device=dev,
                             n_games=n_games, precision=precision, seed=seed,
                             timeout_thresh=timeout_thresh, win_score=win_score)
            _evaluators[key] = ev
        return ev


def genomes_to_device(individuals, genes: int, ev: D.Evaluator) -> torch.Tensor:
    """Pack a list of genomes (lists of floats) into a [n, genes] device tensor.

    Longer genomes are truncated to the genes the network uses (numpy_nn.py:65-67
    only warns); shorter ones fail like numpy_nn's reshape (numpy_nn.py:63).
    """
    n = len(individuals)
    host = np.empty((n, genes), dtype=np.float64)
    for r, ind in enumerate(individuals):
        if len(ind) < genes:
            raise ValueError(f"cannot reshape array of size {len(ind)} into the network's {genes} genes "
                             f"(individual {r})")
        host[r] = np.asarray(ind[:genes], dtype=np.float64)
    return torch.from_numpy(host).to(device=ev.device, dtype=ev.dtype)
