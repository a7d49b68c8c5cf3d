timeout -k 10 300 python -m pytest tests/test_gpu_resize.py -x -q -m gpu > gpurun_out/t_resize.log 2>&1 || { echo TESTFAIL; exit 1; }
export FILTERS=1,4 B=32
FLUSH=,2,3 BANDS=,16,32 timeout -k 10 300 python tools/sweep_resize.py > gpurun_out/sweep_f.log 2>&1
