"""Per-parameter gradient differences of one training step with and without
the fused BN backward reduces (ops.FUSE_BN_REDUCE), to locate where they first
appear (diagnostic; GPU)."""
import itertools
import sys

import torch

sys.path.insert(0, "audio-training_amd")
sys.path.insert(0, ".")
from acfe import ops  # noqa: E402
from acfe.train import FrontEnd, Trainer  # noqa: E402
import bench  # noqa: E402

BF = torch.bfloat16
cuda = torch.device("cuda:0")
name = sys.argv[1] if len(sys.argv) > 1 else "bird"
outs = []
for fuse in (False, True):
    ops.FUSE_BN_REDUCE = fuse
    torch.manual_seed(0)
    if name == "bird":
        from resnet.wr_resnet_bird import WRResNet
        model = WRResNet(input_shape=(128, 513, 3), classes=10, dtype=BF).to(cuda)
    else:
        from resnet.wr_resnet import WRResNet
        model = WRResNet(input_shape=(128, 513, 1), classes=10, dtype=BF).to(cuda)
    fe = FrontEnd(n_mels=128, dtype=BF, device=cuda).to(cuda)
    tr = Trainer(model, fe, lr=0.0, loss="cce", device=cuda)
    x1, x2, lam, y = bench.make_batches(4, 10, cuda, n_sets=1)[0]
    ops._seed_counter = itertools.count()
    loss, z = tr.step(x1, y, x2, lam)
    torch.cuda.synchronize()
    names = [n for n, p in tr.holder.named_parameters() if p.requires_grad]
    outs.append([(n, tr.arena.grad[o:o + k].detach().double().clone()) for n, (o, k) in zip(names, tr.arena.offsets)])
for (n, a), (_, b) in zip(*outs):
    d = (b - a).norm().item()
    r = d / max(a.norm().item(), 1e-30)
    print(f"{r:10.3e} {a.norm().item():10.3e} {n}")
