set -u
export TMPDIR=/tmp SWEEP_CB=/tmp/sweep_cb.npz SWEEP_REPS=3
mkdir -p gpurun_out/r2_st1
timeout -k 10 300 python tools/screen_sweep.py > gpurun_out/r2_st1/sweep.log 2>&1 || { tail gpurun_out/r2_st1/sweep.log; exit 1; }
tail -1 gpurun_out/r2_st1/sweep.log
RQSID_SCREEN_VARIANT=6 RQSID_LIB=tools/ab/librqsid_ab0.so timeout -k 10 300 python tools/res_stamps.py > gpurun_out/r2_st1/stamps.log 2>&1 || { tail gpurun_out/r2_st1/stamps.log; exit 1; }
cat gpurun_out/r2_st1/stamps.log
