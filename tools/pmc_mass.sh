#!/bin/bash
# PMC passes of the C3 mass inverse kernels (tools/pmc_mass_child.py), one
# rocprofv3 run per pass, no tracing domain beside --pmc:  tools/pmc_mass.sh TAG
TAG=${1:-pmc_mass}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o pmc -- python tools/pmc_mass_child.py > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $p"
  if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
