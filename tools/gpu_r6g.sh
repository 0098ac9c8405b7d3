O=gpurun_out/${1:-r6g}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_advbas.py tests/test_bfcp.py tests/test_cabi.py tests/test_comm.py tests/test_device_helpers.py tests/test_gpu_determinism.py tests/test_gpu_factor.py tests/test_gpu_lp.py -m gpu -k "not sharded and not rccl and not comm" > $O/v_revert.log 2>&1
echo "rc $?" >> $O/v_revert.log
