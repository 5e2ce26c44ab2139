#!/bin/bash
# PMC counter passes for the stencil kernel (one rocprofv3 run per pass;
# no tracing domains combined with --pmc).  Usage: tools/pmc_stencil.sh TAG [bench args]
TAG=${1:-pmc}; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
ARGS="--pmc-child $*"
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o pmc -- python bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $p"
  if [ $rc -gt 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT"
