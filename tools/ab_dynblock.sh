# tier workgroups of 512 lanes (default) vs 1024 on the same (1024-costed) plan
export TMPDIR=/tmp
for cfg in 2 3 4; do
  for v in "" "RAOCP_DYN_BLOCK=1024" ""; do
    echo -n "c$cfg [$v] "
    env $v timeout -k 10 120 python3 tools/prof_cp.py $cfg 240 2>&1 | tail -1 || exit 1
  done
done
