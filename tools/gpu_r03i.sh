# Kernel traces of eager dynamics projections (tiers and the per-stage sweep) at configs 2,
# 4 and 5: per-launch durations and gaps (tools/trace_seq.py).
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
run() {  # tag config env...
  local tag=$1 cfg=$2; shift 2
  env "$@" RAOCP_DYN_VERBOSE=1 timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tr_$tag -o tr --output-format csv -- python3 tools/dyn_trace.py $cfg 20 > gpurun_out/tr_$tag.log 2>&1 || { echo "trace $tag failed"; tail -5 gpurun_out/tr_$tag.log; return 1; }
  python3 tools/trace_seq.py gpurun_out/tr_$tag 48 > gpurun_out/seq_$tag.log && echo "== $tag" && grep -E "plan|x[0-9]" gpurun_out/tr_$tag.log | head -3 && cat gpurun_out/seq_$tag.log
}
run c2_tiers 2 RAOCP_DYN3=0 && run c4_tiers 4 RAOCP_DYN3=0 && run c4_dy3 4 RAOCP_DYN3=1 && run c2_dy3 2 RAOCP_DYN3=1 && run c5_dy3 5 RAOCP_DYN3=1
