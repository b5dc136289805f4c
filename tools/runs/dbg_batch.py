# development: the native batch (sa_align_batch) against the reference's batch records
import sys, os
sys.path[:0] = [os.getcwd() + "/sequence-alignment-gpu_amd/python", os.getcwd() + "/oracle", os.getcwd() + "/tests"]
from sa_amd import engine, synthetic
import oracle
from test_batch_golden import fixture, inputs, record
doc = fixture()
count = int(sys.argv[1]) if len(sys.argv) > 1 else 512
pairs = [inputs("global", i) for i in range(count)]
got = engine.align_batch(0, [t for t, _ in pairs], [p for _, p in pairs], synthetic.blast_matrix(), doc["gap"], num_gpus=1)
bad = [i for i in range(count) if record(got[i]) != doc["global"]["records"][i]]
print("count", count, "bad", len(bad))
for i in bad[:2]:
    print(i, record(got[i]), doc["global"]["records"][i])
    o = oracle.align(0, pairs[i][0], pairs[i][1], synthetic.blast_matrix(), doc["gap"])
    r = got[i]
    print("   oracle", {k: o[k] for k in ("score", "num_bytes", "start_text", "start_pattern")}, "strings equal:", o["aligned_text"] == r["aligned_text"], o["aligned_pattern"] == r["aligned_pattern"])
