# round 6: r06_b2 (tests + config-5 shard sweep) then r06_b3 (tail strip groups A/B + timelines, pair
# fill priority A/B), one box
bash tools/runs/r06_b2.sh && bash tools/runs/r06_b3.sh
