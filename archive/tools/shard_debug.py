"""Locate the first mismatch of the simulated sharded sequence vs single-GPU."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import numpy as np
import kltamd
from conftest import synth
from kltabi import OracleTracker, load_oracle
from test_shard import sharded_sequence
from kltamd.shard import band_of

gpu = kltamd.load(); gpu.KLTSetVerbosity(0)
world, chunk, margin = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
frames = synth(gpu, 2160 + world, 640, 480, 11)
orc = OracleTracker(load_oracle())
X, Y, V = orc.harness(frames, 1500, 11, first=frames[0])
for T in range(2, 12):
    x, y, v, redone = sharded_sequence(gpu, frames[:T], 1500, world, chunk, margin)
    k = T - 2
    bad = np.nonzero((v != V[:, k]) | (x.view(np.int32) != X[:, k].view(np.int32)) | (y.view(np.int32) != Y[:, k].view(np.int32)))[0]
    print("frames", T, "redone", redone, "mismatches", len(bad))
    if len(bad):
        for f in bad[:10]:
            prev = (X[f, k - 1], Y[f, k - 1], V[f, k - 1]) if k > 0 else None
            print(f"  f{f}: got ({x[f]}, {y[f]}, {v[f]}) want ({X[f,k]}, {Y[f,k]}, {V[f,k]}) prev {prev}")
        print([band_of(480, world, r, margin) for r in range(world)])
        break
