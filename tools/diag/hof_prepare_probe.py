#!/usr/bin/env python3
"""Time the device steps of DeviceGA._hof_update's prepare phase at config-4
sizes (131 072 members, k candidates of 524 288 rows), each alone with HIP
events: where the ~1.8 ms go.  usage: python tools/diag/hof_prepare_probe.py [k]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "neuro-genetic-pong-self-play_amd"))
from pong_amd import device as D  # noqa: E402

dev = torch.device("cuda", 0)
P, H, G = 524288, 131072, 643
k = int(sys.argv[1]) if len(sys.argv) > 1 else 15000
gen = torch.Generator(device=dev).manual_seed(1)
rows = torch.randn((P, G), generator=gen, dtype=torch.float64, device=dev)
fit = torch.randn(P, generator=gen, dtype=torch.float64, device=dev)
hof_fit = torch.sort(torch.randn(H, generator=gen, dtype=torch.float64, device=dev), descending=True).values
hof_hash = torch.randint(0, 1 << 62, (H,), generator=gen, device=dev)
worst = float(torch.sort(fit, descending=True).values[k])


def t(name, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        out = fn()
    b.record()
    torch.cuda.synchronize()
    res[name] = a.elapsed_time(b) / reps
    return out


res = {}
cand = t("nonzero", lambda: torch.nonzero(fit > worst).flatten())
kk = int(cand.numel())
h = t("row_hash", lambda: D.row_hash(rows, G, index=cand.to(torch.int32)))
fc = t("gather_fit", lambda: fit[cand])
n = H + kk
by_age = t("cat_flip", lambda: torch.cat([hof_fit.flip(0), fc]))
order = t("sort_stable", lambda: torch.sort(by_age, stable=True).indices)


def rank_fn():
    ra = torch.empty_like(order)
    ra[order] = torch.arange(n, device=dev)
    return torch.cat([ra[:H].flip(0), ra[H:]])


rank = t("rank_scatter", rank_fn)
hashes = t("cat_hash", lambda: torch.cat([hof_hash, h]))
cls = t("unique_inverse", lambda: torch.unique(hashes, return_inverse=True)[1])
packed_d = t("pack", lambda: torch.cat([rank | (cls << 32), fc.view(torch.int64)]))
packed_h = torch.empty(packed_d.shape, dtype=torch.int64, pin_memory=True)
t("d2h", lambda: packed_h.copy_(packed_d, non_blocking=True))
res["k"] = kk
res["total_ms"] = sum(v for key, v in res.items() if key not in ("k",))
print(json.dumps(res))
