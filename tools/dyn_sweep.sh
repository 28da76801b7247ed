# dynamics engine / tier-plan sweep: CP it/s at configs 2, 3, 4
export TMPDIR=/tmp
for cfg in 4 3 2; do
  for v in "" "RAOCP_DYN_PER_STAGE=1" "RAOCP_DYN_CUT=1" "RAOCP_DYN_CUT=2" "RAOCP_DYN_CUT=3" "RAOCP_DYN_CUT=4" "RAOCP_DYN_FOLD=1" "RAOCP_CP_V1=1"; do
    echo -n "c$cfg [$v] "
    env $v timeout -k 10 120 python3 tools/prof_cp.py $cfg 480 2>&1 | tail -1 || exit 1
  done
done
