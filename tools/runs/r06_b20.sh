# round 6: one-shot calls stage through the pinned buffer with a copy kernel instead of DMA copies
# (SA_STAGE_KERNEL): the tests that go through sa_align_pair, then the harness latency mode A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_edge_cases.py tests/test_cli.py tests/test_ref_callers.py tests/test_harness.py tests/test_capi.py > gpurun_out/r6b20_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b20_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b20_tests.log
mkdir -p gpurun_out/r6b20_cwd
python tools/score_matrices.py gpurun_out/r6b20_cwd || exit 1
bin=$PWD/sequence-alignment-gpu_amd/bin/sa_benchmarks
out=$PWD/gpurun_out/r6b20.log
: > $out
cd gpurun_out/r6b20_cwd || exit 1
for rep in 1 2; do
  for sk in 1 0; do
    echo "== SA_STAGE_KERNEL=$sk latency global" >> $out
    SA_STAGE_KERNEL=$sk timeout -k 10 240 $bin latency global --repeats 5 --json >> $out 2>&1 || exit 1
    echo "== SA_STAGE_KERNEL=$sk latency local" >> $out
    SA_STAGE_KERNEL=$sk timeout -k 10 240 $bin latency local --repeats 5 --json >> $out 2>&1 || exit 1
  done
done
grep "==\|\"latency\"" $out | cut -c1-150
