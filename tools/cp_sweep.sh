# CP block-shape sweep: it/s at configs 2 and 4 for family / leaf block sizes (env overrides)
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in 4 2; do
for lb in default 64 32 16 8; do
  for fb in default 4 2; do
    env_lb=""; env_fb=""
    [ "$lb" != default ] && env_lb="RAOCP_CP_LB=$lb"
    [ "$fb" != default ] && env_fb="RAOCP_CP_FB=$fb"
    echo -n "c$cfg LB=$lb FB=$fb: "
    env $env_lb $env_fb timeout -k 10 120 python3 tools/prof_cp.py $cfg 480 2>&1 | tail -1 || exit 1
  done
done
done
