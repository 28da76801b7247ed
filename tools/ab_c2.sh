# A/B timing of dynamics / stopping-test switches at config 2 (CP us/it) and the dynamics
# stamps with and without rotated staging
export TMPDIR=/tmp
for v in "" "RAOCP_DYN_ROT=0" "RAOCP_DEFER_CHECK=0" "RAOCP_DYN_ROT=0 RAOCP_DEFER_CHECK=0"; do
  echo -n "c2 [$v] "
  env $v timeout -k 10 120 python3 tools/prof_cp.py 2 960 2>&1 | tail -1 || exit 1
done
for v in "" "RAOCP_DYN_ROT=0"; do
  echo "stamps [$v]"
  env $v timeout -k 10 120 python3 tools/stamps.py 2 2>&1 | tail -6 || exit 1
done
