"""The device's f64 forward in numpy's exact operation order (run with -m gpu).

numpy_nn.run computes each layer as np.dot(w, column) (numpy_nn.py:127): an
OpenBLAS dgemv_t with its own summation order (oracle/pong_oracle.c
or_blas_dot, pinned to np.dot by tests/test_blas_order.py), then the sigmoid
1 / (1 + np.e ** -z) (numpy_nn.py:22-23).  Here every layer's pre-activations
of pg_forward's f64 path must equal the restated np.dot of the device's own
inputs to that layer bit for bit, and every activation the correctly rounded
sigmoid (pg_f64math.h compiled for the host).  pg_decide -- the hot kernel's
decision cascade -- must equal the f64 argmax everywhere.
"""
import os
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "neuro-genetic-pong-self-play_amd", "csrc", "pg_f64math.h")


def _gene_count(shape, bias=True):
    b = 1 if bias else 0
    return sum((shape[i] + b) * shape[i + 1] for i in range(len(shape) - 1))


def _host_sigmoid(tmp_path, z):
    src = tmp_path / "s.c"
    src.write_text(f'#include <stdio.h>\n#include "{HDR}"\n'
                   "int main(void){ double z; while (scanf(\"%la\", &z) == 1) "
                   "printf(\"%a\\n\", pg_sigmoid_f64(z)); return 0; }\n")
    exe = tmp_path / "s"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"])
    out = subprocess.run([str(exe)], input="\n".join(float(v).hex() for v in z), capture_output=True, text=True,
                         check=True).stdout.split()
    return np.array([float.fromhex(v) for v in out])


@pytest.mark.parametrize("shape,bias,n_gen", [
    ([6, 64, 3], True, 64), ([6, 2, 2], True, 64), ([6, 8, 8, 3], True, 32), ([6, 7, 5, 2], True, 32),
    ([6, 4, 2], False, 32), ([6, 3000, 2], True, 2), ([6, 512, 512, 3], True, 2)])
def test_f64_layers_in_numpy_order(gpu, oracle, tmp_path, shape, bias, n_gen):
    from pong_amd.device import Evaluator
    rng = np.random.default_rng(sum(shape) + (0 if bias else 7))
    G = _gene_count(shape, bias)
    genes = rng.standard_normal((n_gen, G)) * 3.0
    per = 8
    n = n_gen * per
    gi = np.repeat(np.arange(n_gen), per).astype(np.int32)
    x = rng.integers(0, 321, size=(n, 6)) * 0.5 / 160.0
    ev = Evaluator(shape, bias=bias, device=gpu, precision="f64")
    idx, act = ev.forward(torch.tensor(genes, device=gpu), torch.tensor(x, device=gpu),
                          genome_index=torch.tensor(gi, device=gpu), want_layers=True)
    z_all, h_all = (t.cpu().numpy() for t in ev.last_layers)
    b = 1 if bias else 0
    zs = []
    for t in range(n):
        g = genes[gi[t]]
        inp = np.append(x[t], 1.0) if bias else x[t]
        off, u = 0, 0
        for l in range(len(shape) - 1):
            nin, nout = shape[l], shape[l + 1]
            w = g[off:off + (nin + b) * nout].reshape(nout, nin + b)
            want = oracle.blas_gemv(w, inp)
            np.testing.assert_array_equal(z_all[t, u:u + nout], want, err_msg=f"pass {t} layer {l}")
            zs.append(z_all[t, u:u + nout])
            h = h_all[t, u:u + nout]
            inp = np.append(h, 1.0) if bias else h
            off += (nin + b) * nout
            u += nout
    z_cat = np.concatenate(zs)
    np.testing.assert_array_equal(h_all.reshape(-1), _host_sigmoid(tmp_path, z_cat))
    # np.argmax of the device's own output activations
    last = shape[-1]
    np.testing.assert_array_equal(idx.cpu().numpy(), np.argmax(h_all[:, -last:], axis=1))


@pytest.mark.parametrize("shape", [[6, 64, 3], [6, 2, 2], [6, 16, 4], [6, 100, 3], [6, 200, 2]])
def test_decide_cascade_equals_f64(gpu, shape):
    """pg_decide (k_service's cascade: f32 certificate, plateau rules, the
    frame's own bound, certified f64, numpy-order f64) == the all-f64 forward's argmax on 300k+ decisions,
    incl. the saturation-heavy N(0, 9) / N(0, 30) regimes."""
    from pong_amd.device import Evaluator
    rng = np.random.default_rng(shape[1] * 7 + shape[2])
    G = _gene_count(shape)
    ev = Evaluator(shape, device=gpu)
    stages = np.zeros(5, np.int64)
    for sigma in (1.0, 3.0, 9.0, 30.0):
        n_gen, per = 512, 160
        genes = torch.tensor(rng.standard_normal((n_gen, G)) * sigma, device=gpu)
        gi = torch.tensor(np.repeat(np.arange(n_gen), per), dtype=torch.int32, device=gpu)
        k = rng.integers(0, 321, size=(n_gen * per, 6)).astype(np.int32)
        idx, stage = ev.decide(genes, torch.tensor(k, device=gpu), genome_index=gi)
        x = torch.tensor(k * 0.5 / 160.0, device=gpu)
        ref, _ = ev.forward(genes, x, genome_index=gi, precision="f64", want_act=False)
        np.testing.assert_array_equal(idx.cpu().numpy(), ref.cpu().numpy())
        stages += np.bincount(stage.cpu().numpy(), minlength=5)
    print(f"shape {shape}: decision stages {stages.tolist()} (f32, in-wave plateau, service certified, numpy-order, "
          "frame bound)")
    assert stages[0] > 0.9 * stages.sum()
    if shape[1] > 32 and shape[1] <= 64:  # serve_inline's layout (L = 8, U = 16): the frame bound's tier runs
        assert stages[4] > 0
