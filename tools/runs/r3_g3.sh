# round 3, call g3: the GPU suite on the certify change, per-phase generation profile at P = 524 288 and 65 536
# (fused generation path), and the wide kernel's stream rate with f32 vs f64
# genomes (per-frame working set 0.27 vs 0.54 GB of W2 copies beside the
# 256 MB Infinity Cache)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_g3}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ga_profile.py 524288 8 > $OUT/ga_profile_524k.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/ga_profile.py 65536 8 > $OUT/ga_profile_65k.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --pop 16384 --dtype f32 > $OUT/wide_f32.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 0 --reps 2 --kernel wide --shape 6,512,512,3 --pop 16384 --dtype f64 > $OUT/wide_f64.log 2>&1 || exit 1
echo done > $OUT/ok
