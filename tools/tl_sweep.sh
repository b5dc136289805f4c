set -o pipefail
mkdir -p gpurun_out
for c in "64 4" "256 4" "1024 4" "32768 4" "32768 2" "32768 1"; do set -- $c
  echo "== m=$1 waves=$2" >> gpurun_out/tl.log
  timeout -k 10 60 python tools/timeline.py --n 32768 --m $1 --waves $2 >> gpurun_out/tl.log 2>&1 || exit 1
done
