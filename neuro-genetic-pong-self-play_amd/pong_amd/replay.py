"""Replays of evaluated games: what the reference's render path shows
(evaluate(render=True) -> render_game main.py:115-125, used by
pickle_inspector.py), headless.

A genome's games are played once by pg_eval_population with per-frame action
traces; the traced actions are then stepped again through the SoA stepper
(pg_physics_step) and every frame is rasterised on the device
(pg_render_frames).  The reference shows the frames in a gym viewer at FPS;
here they are returned as arrays and can be written as animated GIFs.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from . import device as D

_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def game_seed(base: int, game: int) -> int:
    """Physics seed of game slot ``game`` (csrc/pg_device.hpp game_seed)."""
    return _splitmix64((base ^ ((0xA24BAED4963EE407 * (game + 1)) & _M64)) & _M64)


def _code_bits(code: np.ndarray, shift: int) -> np.ndarray:
    # action code 1 = [1, 0] (up), 2 = [0, 1] (down) -> pg_physics_step bits
    return (((code == 1).astype(np.uint8)) | ((code == 2).astype(np.uint8) << 1)) << shift


def replay(ev: D.Evaluator, genome: torch.Tensor, kind, opp, mult, opponents: Optional[torch.Tensor] = None,
           cap: int = 8192, every: int = 1):
    """Play one genome's games with traces and re-render them.

    Returns (EvalResult, frames): frames[g] is a uint8 array [F_g / every, 210,
    160, 3] of game g's frames (after each env.step).  The re-simulated final
    scores are checked against the evaluation's."""
    dev = ev.device
    games = ev.n_games
    kind_t = torch.as_tensor(np.asarray(kind, np.int32).reshape(1, games), device=dev)
    opp_t = torch.as_tensor(np.asarray(opp, np.int32).reshape(1, games), device=dev)
    mult_t = torch.as_tensor(np.asarray(mult, np.float64).reshape(1, games), device=dev)
    res, trace = ev.evaluate(genome.reshape(1, -1).contiguous(), kind_t, opp_t, mult_t, opponents=opponents,
                             trace_games=games, trace_cap=cap)
    frames_n = res.frames[0].cpu().numpy()
    if frames_n.max() > cap:
        raise ValueError(f"a game ran {frames_n.max()} frames; raise cap above that")
    tr = trace.cpu().numpy()
    ph = D.Physics(games, device=dev)
    seeds = torch.tensor([game_seed(ev.seed, g) - (1 << 64) if game_seed(ev.seed, g) >= 1 << 63
                          else game_seed(ev.seed, g) for g in range(games)], dtype=torch.int64, device=dev)
    ph.reset(seeds, (kind_t[0] == 1).to(torch.int32).contiguous())
    out = [[] for _ in range(games)]
    ends = set(frames_n.tolist())
    for t in range(1, int(frames_n.max()) + 1):
        # env.step at frame t applies the decision traced at frame t - 1 (none at frame 1)
        prev = tr[:, t - 2] if t >= 2 else np.zeros(games, np.uint8)
        act = _code_bits(prev & 3, 0) | _code_bits((prev >> 2) & 3, 2)
        ph.step(torch.as_tensor(act, device=dev))
        if (t - 1) % every == 0:
            img = D.render_frames(ph.state).cpu().numpy()
            for g in range(games):
                if t <= frames_n[g]:
                    out[g].append(img[g])
        if t in ends:
            s = ph.fields()
            for g in np.nonzero(frames_n == t)[0]:
                got = (int(s["score1"][g]), int(s["score2"][g]))
                want = tuple(int(v) for v in res.scores[0, g].cpu().numpy())
                if got != want:
                    raise RuntimeError(f"replay of game {g} ended at {got}, the evaluation at {want}")
    return res, [np.stack(f) if f else np.zeros((0, 210, 160, 3), np.uint8) for f in out]


def write_gif(frames: np.ndarray, path: str, fps: int = 60) -> str:
    """An animated GIF of a [T, 210, 160, 3] frame stack (the viewer's FPS, config.FPS)."""
    from PIL import Image
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    imgs = [Image.fromarray(f) for f in frames]
    imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=max(1, int(1000 / fps)), loop=0)
    return path
