# round-5 check 12: why the native batch results differ (test_batch_abi global-512-1)
mkdir -p gpurun_out
echo "--- head"; timeout -k 10 120 python tools/runs/dbg_batch.py 256 2>&1 | grep -v amdgpu.ids | head -3
echo "--- head, unpacked fill"; SA_NO_PAIR16=1 timeout -k 10 120 python tools/runs/dbg_batch.py 256 2>&1 | grep -v amdgpu.ids | head -3
echo "--- head, generic walk"; SA_TB_GENERIC=1 timeout -k 10 120 python tools/runs/dbg_batch.py 256 2>&1 | grep -v amdgpu.ids | head -3
echo "--- base0"; SA_HIP_LIB=$PWD/build_exp/libsa_base0.so timeout -k 10 120 python tools/runs/dbg_batch.py 256 2>&1 | grep -v amdgpu.ids | head -3
