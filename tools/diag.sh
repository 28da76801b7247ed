export TMPDIR=/tmp
timeout -k 10 120 python tools/stamps.py 2 > gpurun_out/d_stamps.txt 2>&1 && \
timeout -k 10 120 python tools/stamps_cpp.py > gpurun_out/d_cpp.txt 2>&1 && \
timeout -k 10 120 python tools/stamps_ell.py > gpurun_out/d_ell.txt 2>&1 && \
timeout -k 10 120 python tools/roles.py 2 > gpurun_out/d_roles.txt 2>&1
echo rc=$?
cat gpurun_out/d_*.txt
