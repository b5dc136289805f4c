# round-5 check 25: tb_table_kernel phase times (SA_TB_TABLE_TIMING), global / local 32768^2, 8192^2
set -o pipefail
timeout -k 10 120 python tools/tb_table_timing.py --mode 0 > gpurun_out/b25.log 2>&1 || { tail gpurun_out/b25.log; exit 1; }
timeout -k 10 120 python tools/tb_table_timing.py --mode 1 >> gpurun_out/b25.log 2>&1 || { tail gpurun_out/b25.log; exit 1; }
timeout -k 10 120 python tools/tb_table_timing.py --mode 0 --n 8192 --m 8192 >> gpurun_out/b25.log 2>&1 || { tail gpurun_out/b25.log; exit 1; }
grep '^{' gpurun_out/b25.log
