"""Write the reference's score-matrix text files (scoreMatrices/<dna|protein>/<name>.txt, whitespace
separated rows, the format parseScoreMatrixFile reads) into a directory, from the committed
tests/golden/matrices.json. The CLI and sa_benchmarks load their default matrices by that relative
path (include/SequenceAlignment.hpp DEFAULT_*_SCORE_MATRIX_FILE), so they run from such a directory.

    python tools/score_matrices.py <dir>
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def write(dest: str) -> None:
    mats = json.load(open(os.path.join(ROOT, "tests", "golden", "matrices.json")))
    for name, v in mats.items():
        A = 4 if len(v) == 16 else 23
        sub = "dna" if A == 4 else "protein"
        os.makedirs(os.path.join(dest, "scoreMatrices", sub), exist_ok=True)
        with open(os.path.join(dest, "scoreMatrices", sub, f"{name}.txt"), "w") as f:
            f.write("\n".join(" ".join(str(x) for x in v[r * A:(r + 1) * A]) for r in range(A)) + "\n")


if __name__ == "__main__":
    write(sys.argv[1] if len(sys.argv) > 1 else ".")
