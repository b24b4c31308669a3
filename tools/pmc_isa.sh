#!/bin/bash
# Real cycles per VALU wave-instruction of each microbenchmarked opcode (tools/microbench/isa_rate4):
# GRBM_GUI_ACTIVE (summed over the 8 XCDs) against SQ_INSTS_VALU, one --pmc pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_isa}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES \
  -d $OUT/p1 -o pmc --output-format csv -- ./tools/microbench/isa_rate4 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
python3 tools/pmc_summary.py $OUT > /dev/null
python3 - "$OUT" <<'PY'
import json, sys, re
d = json.load(open(sys.argv[1] + "/summary.json"))
for k, v in d.items():
    name = re.sub(r".*thr<([^>]*)>.*", r"\1", k)
    cyc = v["GRBM_GUI_ACTIVE"] / 8.0            # per XCD
    per_simd = v["SQ_INSTS_VALU"] / 1024.0      # 256 CUs x 4 SIMDs
    print(f"{name:12s} real cycles per wave-instr per SIMD: {cyc / per_simd:6.2f}   VALUBusy-formula {100*v['SQ_ACTIVE_INST_VALU']/256/cyc:6.1f} %")
PY
