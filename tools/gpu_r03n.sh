# Round-3 final profiles: rocprofv3 statistics + PMC traffic of the bench, tiered-sweep stamps,
# per-stage sweep traces (tools/gpu_r03g.sh, tools/gpu_r03m.sh) and the ASan driver.
export TMPDIR=/tmp
set -o pipefail
rm -rf gpurun_out/r03_prof gpurun_out/pmc2_FETCH_SIZE gpurun_out/pmc2_WRITE_SIZE
bash tools/gpu_r03g.sh && bash tools/gpu_r03m.sh
