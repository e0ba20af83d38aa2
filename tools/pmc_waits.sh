#!/bin/bash
# What k_service's waves wait on: two SQ counter passes over tools/sweep.py's
# one-launch workload (the same as tools/pmc_sq.sh): waits for LDS, the
# instruction fetch, the outstanding LDS / scalar / vector memory levels, LDS
# bank conflicts.  usage: tools/pmc_waits.sh TAG
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd); export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM"
P2="SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_LDS SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/$OUT/p$i -o pmc -- python3 $ROOT/tools/sweep.py --one --lane=8 --reps 1 > $OUT/p$i.out 2> $OUT/p$i.err
  rc=$?; echo "pass $i exit=$rc" >> $OUT/summary.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
python3 - $OUT <<'PY' >> $OUT/summary.txt
import collections, csv, json, sys
d = {}
steps = None
for p in ("p1", "p2"):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{sys.argv[1]}/{p}/pmc_counter_collection.csv")):
        if "k_service" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        d[k] = v[-1]
    try:
        steps = json.loads(open(f"{sys.argv[1]}/{p}.out").read().strip().splitlines()[-1])["env_steps"]
    except Exception:
        pass
wc = d["SQ_WAVE_CYCLES"]
print("stepped env-steps", steps)
print("wave-cycle shares: wait_any %.3f wait_inst_any %.3f wait_inst_lds %.3f" % (
    d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_WAIT_INST_LDS"] / wc))
print("outstanding per wave-cycle: LDS %.3f SMEM %.3f VMEM %.3f IFETCH %.3f" % (
    d["SQ_INST_LEVEL_LDS"] / wc, d["SQ_INST_LEVEL_SMEM"] / wc, d["SQ_INST_LEVEL_VMEM"] / wc, d["SQ_IFETCH_LEVEL"] / wc))
print("instruction fetches per env-step %.3f; SMEM instructions per env-step %.3f; LDS per env-step %.3f" % (
    d["SQ_IFETCH"] / steps, d["SQ_INSTS_SMEM"] / steps, d["SQ_INSTS_LDS"] / steps))
print("cycles: SMEM %.3f VMEM_RD %.3f of wave-cycles; LDS bank conflicts per LDS instruction %.3f" % (
    d["SQ_INST_CYCLES_SMEM"] / wc, d["SQ_INST_CYCLES_VMEM_RD"] / wc, d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_INSTS_LDS"], 1)))
print(json.dumps(d))
PY
