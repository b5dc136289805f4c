for w in 1 2 4; do
  SA_WAVES_PER_GROUP=$w timeout -k 10 60 python tools/timeline.py --n 32768 --m 256 --waves $w > gpurun_out/tlw2_$w.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/tlw2_$w.json'))
print('W=$w', d['ns_per_step_by_strip'], d['clk_per_step_mean'], d['cu_se_of_first_8'], d['xcc_of_first_16'])"
done
