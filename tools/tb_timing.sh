set -e
cd /root/repo
mkdir -p gpurun_out
for a in "--n 32768 --m 32768 --mode 0" "--n 32768 --m 32768 --mode 1" "--n 8192 --m 8192 --mode 0" "--n 4096 --m 4096 --mode 1"; do
  timeout -k 10 120 python tools/tb_timing.py $a
done
