# Kernel traces of the per-stage sweep with table images at configs 4 and 5.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
run() {  # tag config env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tr_$tag -o tr --output-format csv -- python3 tools/dyn_trace.py $cfg 20 > gpurun_out/tr_$tag.log 2>&1 || { echo "trace $tag failed"; tail -5 gpurun_out/tr_$tag.log; return 1; }
  python3 tools/trace_seq.py gpurun_out/tr_$tag 20 > gpurun_out/seq_$tag.log && echo "== $tag" && cat gpurun_out/seq_$tag.log
}
run c4_img 4 RAOCP_DYN3=1 && run c5_img 5 RAOCP_DYN3=1
