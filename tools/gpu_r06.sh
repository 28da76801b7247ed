# Round-6 GPU runner (one script for every GPU call of the round):
#   gpurun -- 'bash tools/gpu_r06.sh <tag> <step> [<step> ...]'
# Steps run in order, each under its own time limit, output under gpurun_out/<tag>/; the
# first failing step ends the call (no GPU step runs after a failure).
#   drc         tests/test_gpu_drc.py (the fused dynamics + CP launch k_drc)
#   drcq        its config-2 parity cases only
#   drcchk      tools/drc_check.py: the fused loop against the pair and the oracle, op / loop times
#   drcvar      tools/drc_check.py for each library in $DRC_LIBS ("default" or build/var/<v>.so)
#   drskew      tools/dr_skew.py: k_dr's per-workgroup stamps (diagnostic variant build/var/diag.so)
#   drlevels    tools/dr_levels.py: per-level stamps of k_dr and of the sweep inside k_drc
#   drcstamps   tools/drc_stamps.py on the diagnostic variant build/var/diag.so (VAR_UNIT=dynr)
#   dynr        tests/test_gpu_dynr.py (the regular-tree sweep)
#   cp4         tests/test_gpu_cp4.py (k_cp4 against k_cp3 and the oracle)
#   cp5         tests/test_gpu_cp5.py (k_cp5 against k_cp3 and the oracle)
#   cp6         tests/test_gpu_cp6.py (k_cp6 against k_cp4, k_cp3 and the oracle)
#   cptests     the CP-kernel test files (cp3, cp4, cp5, fp32)
#   dyntests    the dynamics test files (dynr, dyn_split, dyn3, variants)
#   tests       the whole -m gpu suite
#   rest        the test files in $REST_TESTS (default tests/test_gpu_variants.py)
#   smoke       __graft_entry__.smoke()
#   dyn         dynamics projection timings at config 2 (tools/dyn_time.py, variants in $DYN_VARIANTS)
#   stamps      in-kernel stamps of the regular-tree sweep at config 2 (tools/dr_stamps.py)
#   cp          CP kernel / dynamics / loop timings (tools/cp3_time.py)
#   lsweep      standalone L / L^T at configs 2, 4 (3 buffer sets) and 5 fp32 (2 sets)
#   lsweepvar   the same at configs 4 and 5 for each variant library build/var/<v>.so in $LSWEEP_LIBS
#               (tools/build_var.sh)
#   cp6stamps   k_cp6's in-kernel stamps at config 2 (diagnostic variant build/var/diag.so)
#   dy3trace    per-launch trace of the config-4 / config-5 dynamics (rocprofv3 kernel trace, tools/trace_seq.py)
#   ksweep      tools/k_sweep.py: device / wall time of a benchmark call against K, graphs and eager
#   bench20     bench.py --steps 20 --warmup 5 (the driver's K)
#   bench       bench.py default run
#   prof        rocprofv3 --kernel-trace --stats of bench.py (eager launches)
#   pmc         FETCH_SIZE / WRITE_SIZE passes of the same bench command
#   asan        the host-ASan ABI driver on the GPU
#   sqpmc       SQ counters (wave cycles split into waiting / issue-stalled / issuing, MFMA busy)
#               of 20 eager CP iterations at configs $KPROF_CFGS, one rocprofv3 --pmc pass each
#   kprof       rocprofv3 --kernel-trace --stats of 20 eager CP iterations at configs $KPROF_CFGS
#               (default "4 5"; tools/prof_cp.py), the kernel statistics of each
export TMPDIR=/tmp
set -o pipefail
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
PYT="python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread"
BARGS="--steps 96 --warmup 24 --no-cpu --no-shard --op-reps 200 --fp32-steps 12"
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    drc) timeout -k 10 600 $PYT tests/test_gpu_drc.py > $out/pytest_drc.log 2>&1 || fail $step $out/pytest_drc.log
          tail -3 $out/pytest_drc.log ;;
    drcq) timeout -k 10 300 $PYT tests/test_gpu_drc.py -k "matches_dr_cp6_and_oracle and c2" > $out/pytest_drcq.log 2>&1 || fail $step $out/pytest_drcq.log
          tail -3 $out/pytest_drcq.log ;;
    drcchk) timeout -k 10 240 python -u tools/drc_check.py 30 > $out/drc_check.log 2>&1 || fail $step $out/drc_check.log
          cat $out/drc_check.log ;;
    drcvar) for v in ${DRC_LIBS:-}; do
              if [ "$v" = default ]; then lib=raocp-toolbox_amd/raocp/core/libraocp_hip.so; else lib=build/var/$v.so; fi
              RAOCP_HIP_LIB=$lib timeout -k 10 120 python -u tools/drc_check.py 30 > $out/drc_check_$v.log 2>&1 || fail $step $out/drc_check_$v.log
              echo "variant $v: $(grep -h 'op 11\|loop' $out/drc_check_$v.log | tr '\n' ' ')"
            done ;;
    drskew) RAOCP_HIP_LIB=build/var/diag.so timeout -k 10 120 python -u tools/dr_skew.py 2 5 > $out/dr_skew.log 2>&1 || fail $step $out/dr_skew.log
          cat $out/dr_skew.log ;;
    drlevels) RAOCP_HIP_LIB=build/var/diag.so timeout -k 10 120 python -u tools/dr_levels.py 4 > $out/dr_levels.log 2>&1 || fail $step $out/dr_levels.log
          cat $out/dr_levels.log ;;
    drcstamps) RAOCP_HIP_LIB=build/var/diag.so RAOCP_STAMP_KERNEL=f timeout -k 10 120 python -u tools/drc_stamps.py 6 > $out/drc_stamps.log 2>&1 || fail $step $out/drc_stamps.log
          cat $out/drc_stamps.log ;;
    drcprobe) RAOCP_HIP_LIB=build/var/${PROBE_LIB:-diag}.so timeout -k 10 300 python -u tools/drc_probe.py 400 > $out/drc_probe_${PROBE_LIB:-diag}.log 2>&1 || fail $step $out/drc_probe_${PROBE_LIB:-diag}.log
          cat $out/drc_probe_${PROBE_LIB:-diag}.log ;;
    dynr) timeout -k 10 500 $PYT tests/test_gpu_dynr.py > $out/pytest_dynr.log 2>&1 || fail $step $out/pytest_dynr.log
          tail -3 $out/pytest_dynr.log ;;
    cp4) timeout -k 10 500 $PYT tests/test_gpu_cp4.py > $out/pytest_cp4.log 2>&1 || fail $step $out/pytest_cp4.log
          tail -3 $out/pytest_cp4.log ;;
    cp5) timeout -k 10 600 $PYT tests/test_gpu_cp5.py > $out/pytest_cp5.log 2>&1 || fail $step $out/pytest_cp5.log
          tail -3 $out/pytest_cp5.log ;;
    cp6) timeout -k 10 500 $PYT tests/test_gpu_cp6.py > $out/pytest_cp6.log 2>&1 || fail $step $out/pytest_cp6.log
          tail -3 $out/pytest_cp6.log ;;
    cptests) timeout -k 10 900 $PYT tests/test_gpu_cp3.py tests/test_gpu_cp4.py tests/test_gpu_cp5.py tests/test_gpu_cp6.py tests/test_gpu_fp32.py > $out/pytest_cp.log 2>&1 || fail $step $out/pytest_cp.log
          tail -3 $out/pytest_cp.log ;;
    dyntests) timeout -k 10 900 $PYT tests/test_gpu_dynr.py tests/test_gpu_dyn_split.py tests/test_gpu_dyn3.py tests/test_gpu_variants.py > $out/pytest_dyn.log 2>&1 || fail $step $out/pytest_dyn.log
          tail -3 $out/pytest_dyn.log ;;
    rest) timeout -k 10 900 $PYT ${REST_TESTS:-tests/test_gpu_variants.py} > $out/pytest_rest.log 2>&1 || fail $step $out/pytest_rest.log
          tail -3 $out/pytest_rest.log ;;
    tests) timeout -k 10 1100 $PYT tests > $out/pytest_gpu.log 2>&1 || fail $step $out/pytest_gpu.log
          tail -3 $out/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || fail $step $out/smoke.log
          tail -2 $out/smoke.log ;;
    dyn) timeout -k 10 400 python -u tools/dyn_time.py 2 default ${DYN_VARIANTS:-} > $out/dyn_time.log 2>&1 || fail $step $out/dyn_time.log
          cat $out/dyn_time.log ;;
    stamps) timeout -k 10 200 python -u tools/dr_stamps.py 2 6 > $out/stamps_c2.log 2>&1 || fail $step $out/stamps_c2.log
          cat $out/stamps_c2.log ;;
    cp) timeout -k 10 600 python -u tools/cp3_time.py ${CP_ARGS:-} > $out/cp3_time.log 2>&1 || fail $step $out/cp3_time.log
          cat $out/cp3_time.log ;;
    lsweep) for a in "2 float64 1" "4 float64 3" "5 float32 2"; do
              timeout -k 10 200 python -u tools/l_sweep.py $a >> $out/l_sweep.log 2>&1 || fail $step $out/l_sweep.log
            done; grep config $out/l_sweep.log ;;
    lsweepvar) for v in ${LSWEEP_LIBS:-}; do
                 for a in "4 float64 3" "5 float32 2"; do
                   RAOCP_HIP_LIB=build/var/$v.so timeout -k 10 200 python -u tools/l_sweep.py $a >> $out/l_sweep_$v.log 2>&1 || fail $step $out/l_sweep_$v.log
                 done
                 echo "variant $v"; grep config $out/l_sweep_$v.log
               done ;;
    cp6stamps) for wg in 200 50; do
                 STAMP_WG=$wg RAOCP_HIP_LIB=build/var/diag.so timeout -k 10 120 python -u tools/cp6_stamps.py 3 >> $out/cp6_stamps.log 2>&1 || fail $step $out/cp6_stamps.log
               done; cat $out/cp6_stamps.log ;;
    dy3trace) for cfg in 4 5; do
                timeout -k 10 240 rocprofv3 --kernel-trace -d $out/tr$cfg -o tr --output-format csv -- python3 tools/dyn_time.py child $cfg trace > $out/tr$cfg.log 2>&1 || fail $step $out/tr$cfg.log
                python3 tools/trace_seq.py $out/tr$cfg 30 > $out/dy3_stages_c$cfg.log; cat $out/dy3_stages_c$cfg.log
              done ;;
    ksweep) timeout -k 10 300 python -u tools/k_sweep.py > $out/k_sweep.log 2>&1 || fail $step $out/k_sweep.log
          cat $out/k_sweep.log
          for v in ${KS_LIBS:-}; do
            RAOCP_HIP_LIB=build/var/$v.so KS_EAGER=0 timeout -k 10 300 python -u tools/k_sweep.py > $out/k_sweep_$v.log 2>&1 || fail $step $out/k_sweep_$v.log
            echo "variant $v"; cat $out/k_sweep_$v.log
          done ;;
    bench20) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench_k20.log 2>&1 || fail $step $out/bench_k20.log
          tail -1 $out/bench_k20.log > $out/bench_k20.json; cut -c1-400 $out/bench_k20.json ;;
    bench) timeout -k 10 500 python -u bench.py > $out/bench.log 2>&1 || fail $step $out/bench.log
          tail -1 $out/bench.log > $out/bench.json; cut -c1-400 $out/bench.json ;;
    prof) RAOCP_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py $BARGS > $out/prof.log 2>&1 || fail $step $out/prof.log
          find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/prof_kernel_stats.csv \; ; head -30 $out/prof_kernel_stats.csv ;;
    pmc) for ctr in FETCH_SIZE WRITE_SIZE; do
           timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d $out/pmc_$ctr -o pmc --output-format csv -- python3 bench.py $BARGS > $out/pmc_$ctr.log 2>&1 || fail $step $out/pmc_$ctr.log
         done ;;
    asan) LSAN_OPTIONS=suppressions=tests/asan/lsan.supp timeout -k 10 120 ./build/asan_abi gpu > $out/asan_gpu.log 2>&1 || fail $step $out/asan_gpu.log
          tail -2 $out/asan_gpu.log ;;
    kprof) for cfg in ${KPROF_CFGS:-4 5}; do
             RAOCP_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kprof$cfg -o kp --output-format csv -- python3 tools/prof_cp.py $cfg 20 > $out/kprof$cfg.log 2>&1 || fail $step $out/kprof$cfg.log
             find $out/kprof$cfg -name "*kernel_stats.csv" -exec cp {} $out/kprof${cfg}_stats.csv \; ; echo "config $cfg"; cut -d, -f1-4 $out/kprof${cfg}_stats.csv | head -12
           done ;;
    sqpmc) for cfg in ${KPROF_CFGS:-4 5}; do
             RAOCP_EAGER=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES -d $out/sq$cfg -o sq --output-format csv -- python3 tools/prof_cp.py $cfg 20 > $out/sq$cfg.log 2>&1 || fail $step $out/sq$cfg.log
             python3 tools/sq_summary.py $out/sq$cfg > $out/sq${cfg}_summary.txt 2>&1; head -40 $out/sq${cfg}_summary.txt
           done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
