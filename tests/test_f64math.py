"""The compact f64 sigmoid of the rare re-decision path (csrc/pg_f64math.h),
compiled for the host with gcc, against numpy's 1 / (1 + np.e ** -z)
(numpy_nn.py:22-23) over the whole exp range."""
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "neuro-genetic-pong-self-play_amd", "csrc", "pg_f64math.h")


def test_compact_sigmoid_matches_numpy_within_ulps(tmp_path):
    src = tmp_path / "s.c"
    src.write_text(f'#include <stdio.h>\n#include "{HDR}"\n'
                   "int main(void){ double z; while (scanf(\"%lf\", &z) == 1) printf(\"%.17g\\n\", pg_sigmoid_f64(z)); return 0; }\n")
    exe = tmp_path / "s"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"])
    rng = np.random.default_rng(0)
    z = np.concatenate([rng.uniform(-40, 40, 20000), rng.uniform(-700, 700, 5000), rng.uniform(30, 37, 5000),
                        np.array([0.0, -0.0, 36.7368005696771, 36.73680056967711, -745.0, 709.0, 800.0, -800.0])])
    out = subprocess.run([str(exe)], input="\n".join(repr(float(v)) for v in z), capture_output=True, text=True,
                         check=True).stdout.split()
    got = np.array([float(v) for v in out])
    with np.errstate(over="ignore"):
        ref = 1 / (1 + np.e ** -z)
    ulps = np.abs(got.view(np.int64) - ref.view(np.int64))
    assert ulps.max() <= 4
    assert (ulps == 0).mean() > 0.8
    # exact where it decides ties: saturation at 53 ln 2 and the plateaus below it
    sat = z >= 36.7369
    assert np.all(got[sat] == ref[sat])
