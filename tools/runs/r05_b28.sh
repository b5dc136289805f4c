# round-5 check 28: path deviation from the table windows' centre lines at large sizes
set -o pipefail
timeout -k 10 300 python tools/path_deviation.py --sizes 32768,120000,250000,500000 --mode 0 > gpurun_out/b28.log 2>&1 || { tail gpurun_out/b28.log; exit 1; }
timeout -k 10 300 python tools/path_deviation.py --sizes 32768,120000,250000 --mode 1 --related >> gpurun_out/b28.log 2>&1 || { tail gpurun_out/b28.log; exit 1; }
grep '^{' gpurun_out/b28.log
