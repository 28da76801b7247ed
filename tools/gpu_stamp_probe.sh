# diagnostics: in-kernel stamps and projection times of k_dr at config 2 under cut lists and
# the timing-only RAOCP_DR_FAULT bits (raocp_dynr.h)
export TMPDIR=/tmp
out=gpurun_out/${1:-probe}
mkdir -p $out
shift
for v in "$@"; do
  echo "== $v" >> $out/stamps.log
  env $v timeout -k 10 120 python -u tools/dr_stamps.py 2 4 >> $out/stamps.log 2>&1 || exit 1
  env $v timeout -k 10 120 python -u tools/dyn_time.py 2 default >> $out/stamps.log 2>&1 || exit 1
done
cat $out/stamps.log
