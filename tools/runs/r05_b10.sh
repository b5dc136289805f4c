# round-5 check 10: where the persistent band fill stops paying -- bench lines at 180000^2, 250000^2 and
# 500000^2 with the band fill forced (SA_BAND=1) and off (SA_BAND=0), two steps each
mkdir -p gpurun_out
: > gpurun_out/ab.log
for sz in 180000 250000 500000; do
  for b in 1 0; do
    LABEL=band$b SA_BAND=$b timeout -k 10 300 bash tools/ab.sh -l base -w headline -s 2 -- --size $sz > /dev/null || exit 1
  done
done
cut -c1-120 gpurun_out/ab.log
