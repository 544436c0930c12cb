#!/bin/bash
# PMC passes over tools/alloc_tlb.py --sizes (run on the GPU box from the repo root): does the
# slow-vs-fast allocation difference show in address translation (UTCL1 / UTCL2) or DRAM traffic?
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
cd /tmp || exit 2
sizes="${SIZES:-1,4,8,16,30}"
i=0
for pmc in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum" \
           "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
           "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d /tmp/pa_$i -o run -- \
    python3 "$R/tools/alloc_tlb.py" --sizes "$sizes" --rounds 1 > "$R/gpurun_out/pa_$i.log" 2>&1 || exit 1
  f=$(find /tmp/pa_$i -name "*counter_collection.csv" | head -1)
  cp "$f" "$R/gpurun_out/pa_$i.csv" || exit 1
done
