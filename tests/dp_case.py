"""The data-parallel GPU case shared by tests/test_dp_gpu.py and its rank
processes (tests/dp_gpu_worker.py): the HIP Trainer on wr_resnet_bird (bf16,
dropout 0, eval-mode BatchNormalization -- or training mode with per-replica
statistics --, PCEN on) fed by mix_up pairs of
synthetic 64-frame clips; a global batch of 8 split evenly over the ranks."""
import torch

from conftest import synth_clips

BUCKET_BYTES = 1 << 20      # ~1 MB: several buckets for the 2.3 M-parameter model
GLOBAL_BATCH = 8
N_SAMPLES = 64 * 281        # 64 frames (pad_end): model input 128 x 64
CLASSES = 10


def make_trainer(dev, bucket_bytes=BUCKET_BYTES, training=False):
    """training: BatchNormalization in training mode (per-replica batch
    statistics, MirroredStrategy's non-synced BN) instead of eval mode."""
    from acfe.train import FrontEnd, Trainer
    from resnet.wr_resnet_bird import WRResNet

    torch.manual_seed(0)
    m = WRResNet(input_shape=(128, 64, 3), classes=CLASSES, dtype=torch.bfloat16, dropout=0.0)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():  # non-trivial BN affine / moving statistics
        for name, p in m.named_parameters():
            if name.endswith("gamma"):
                p.copy_(1 + 0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith("beta") or name.endswith("bias"):
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
        for name, b in m.named_buffers():
            if name.endswith("moving_mean"):
                b.copy_(0.1 * torch.randn(b.shape, generator=g))
            elif name.endswith("moving_variance"):
                b.copy_(1 + 0.5 * torch.rand(b.shape, generator=g))
    m = m.to(dev)
    fe = FrontEnd(n_mels=128, dtype=torch.bfloat16, device=dev, pcen=True).to(dev)
    tr = Trainer(m, fe, lr=0.01, loss="cce", device=dev, bucket_bytes=bucket_bytes)
    tr.train(training)  # eval-mode BN: no statistics coupling the clips of a batch
    return tr


def batch(dev, rank=0, world=1):
    """Rank `rank`'s share of the global batch: (x1, x2, lam, mixed labels)."""
    from acfe.train import mix_labels

    x1 = torch.from_numpy(synth_clips(GLOBAL_BATCH, n=N_SAMPLES, seed=101))
    x2 = torch.from_numpy(synth_clips(GLOBAL_BATCH, n=N_SAMPLES, seed=202))
    lam = torch.tensor([0.0, 0.3, 0.9, 0.0, 0.55, 0.0, 0.2, 0.7], dtype=torch.float32)
    y1 = torch.zeros(GLOBAL_BATCH, CLASSES)
    y2 = torch.zeros(GLOBAL_BATCH, CLASSES)
    y1[torch.arange(GLOBAL_BATCH), torch.arange(GLOBAL_BATCH) % CLASSES] = 1
    y2[torch.arange(GLOBAL_BATCH), (3 * torch.arange(GLOBAL_BATCH) + 1) % CLASSES] = 1
    y = mix_labels(y1, y2, lam)
    per = GLOBAL_BATCH // world
    sl = slice(rank * per, (rank + 1) * per)
    return x1[sl].to(dev), x2[sl].to(dev), lam[sl].to(dev), y[sl].to(dev)
