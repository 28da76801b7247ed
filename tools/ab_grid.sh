# L / L^T launch times over the grids (RAOCP_ELL3_GRID / RAOCP_ELLT3_GRID blocks of 256 lanes)
export TMPDIR=/tmp
for v in "RAOCP_ELL3=1" "RAOCP_ELL3_GRID=1024 RAOCP_ELLT3_GRID=1024" "RAOCP_ELL3_GRID=1536 RAOCP_ELLT3_GRID=1536" "RAOCP_ELL3_GRID=3072 RAOCP_ELLT3_GRID=3072" "RAOCP_ELL3_GRID=4096 RAOCP_ELLT3_GRID=4096"; do
  echo "[$v]"
  env $v timeout -k 10 120 python3 tools/l_sweep.py 4 || exit 1
  env $v timeout -k 10 200 python3 tools/l_sweep.py 5 float32 || exit 1
done
