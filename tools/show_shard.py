#!/usr/bin/env python3
"""One line per batch bench JSON (bench.py --workload batch [--shard-of N]): shard, plan, step and fill times."""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    c = d["config"]
    sm = d.get("shard_model", {})
    print(f"{path}: shard_of {sm.get('shard_of', 1)} pairs {d['sample_result']['pairs_per_gpu']} R {c['rows_per_lane']} "
          f"strips {c['strips_per_gpu']} step {d['ms_per_step']} ms fill {d['fill_ms_per_launch']['median']} ms "
          f"tb {d['e2e_ms']['traceback']} ms value {d['value']} GCUPS modelled_N {sm.get('modelled_n_gpu_gcups')} "
          f"pair0 {d['sample_result']['pair0_score']}")
