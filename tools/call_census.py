#!/usr/bin/env python3
"""Census of the C-ABI calls of one T1 training step (wr_resnet_bird, batch
512): every acfe_* entry point the step calls, with its element count and its
HIP-event time on the launch stream.  usage: python tools/call_census.py [B]"""
import collections
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]
import torch  # noqa: E402

import bench  # noqa: E402
from acfe import ops  # noqa: E402
from acfe.train import FrontEnd, Trainer  # noqa: E402
from resnet.wr_resnet_bird import WRResNet  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
model = WRResNet(input_shape=(128, 513, 3), classes=50, dtype=torch.bfloat16).to(dev)
fe = FrontEnd(n_mels=128, dtype=torch.bfloat16, device=dev).to(dev)
tr = Trainer(model, fe, lr=0.01, loss="cce", device=dev)
x1, x2, lam, y = bench.make_batches(B, 50, dev, n_sets=1)[0]
for _ in range(2):
    tr.step(x1, y, x2, lam)
torch.cuda.synchronize()

rec = []
orig = ops.call


def timed(name, *args):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = orig(name, *args)
    e1.record()
    rec.append((name, args, e0, e1))
    return r


ops.call = timed
tr.step(x1, y, x2, lam)
torch.cuda.synchronize()
ops.call = orig
tot = collections.defaultdict(lambda: [0, 0.0])
for name, args, e0, e1 in rec:
    ms = e0.elapsed_time(e1)
    tot[name][0] += 1
    tot[name][1] += ms
    if name.startswith("acfe_bn_") or name.startswith("acfe_add") or name.startswith("acfe_relu"):
        shape = [a for a in args if isinstance(a, int)][:4]
        print(f"  {name:28s} {str(shape):40s} {ms * 1e3:8.1f} us")
print(f"{'entry point':32s} {'calls':>6s} {'ms':>8s}")
for name, (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"{name:32s} {n:6d} {ms:8.3f}")
print(f"total {sum(v[1] for v in tot.values()):.2f} ms")
