#!/usr/bin/env python3
"""Benchmark of the hot path: clips/s of data-parallel TRAINING on synthetic
3 s @ 48 kHz clips (BASELINE.json configs[2]/[3]: wr_resnet_bird, 50 classes,
bf16, batch 512 per GPU, Adam), plus the mel-pipeline GB/s of the fused
front-end kernel.

A step = one pass of the hot path over one batch resident in HBM:
normalize x2 -> mix_up -> normalize -> STFT/|X|^2/mel -> PCEN -> WRN forward
-> loss -> backward -> gradient all-reduce (N > 1) -> Adam.

  python bench.py [--gpus N --steps K --warmup W]
      N > 1: the driver starts it under torch.distributed.run (RANK/WORLD_SIZE
      set); started directly with --gpus N it launches the N ranks itself.
      ACFE_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU (RCCL
      needs one GPU per rank).

Prints ONE JSON line on rank 0.  `roofline` is measured live with HIP events
around the dominant kernel (the forward of the stage-1 block-0 3x3 128->128
convolution, 57 % of the model FLOPs) on the stream it runs on; the rocprofv3
summaries under profiles/ are the cross-check.  `cpu_baseline` times the CPU
restatement of the same step (oracle/, torch-CPU + numpy) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

MI355X_PEAK_BF16_TFLOPS = 2500.0  # dense MFMA (MI355X_MICROARCH.md)
MI355X_PEAK_FP32_TFLOPS = 157.3
MI355X_PEAK_HBM_GBS = 8000.0
N_SAMPLES = 144000
FRONTEND_BYTES_PER_CLIP = 144000 * 4 + 128 * 513 * 4  # SURVEY.md 6 / BASELINE.md 2


def synth_bank(n_clips, seed=20260227, sr=48000, n=N_SAMPLES):
    """SURVEY.md 8(d) synthetic clips: 1-3 linear chirps + white noise, clipped."""
    t = np.arange(n) / sr
    out = np.zeros((n_clips, n), np.float32)
    for i in range(n_clips):
        rng = np.random.default_rng(seed + i)
        x = rng.normal(0, rng.uniform(0.002, 0.02), n)
        if i % 8 != 0:
            for _ in range(rng.integers(1, 4)):
                f0, f1 = rng.uniform(500, 10000, 2)
                amp, on = rng.uniform(0.05, 0.5), rng.uniform(0, 2.0)
                dur = rng.uniform(0.3, 3.0 - on)
                m = (t >= on) & (t < on + dur)
                tt = t[m] - on
                x[m] += amp * np.sin(2 * np.pi * (f0 * tt + 0.5 * (f1 - f0) / dur * tt * tt))
        out[i] = np.clip(x, -1, 1)
    return out


def make_batches(batch, classes, device, n_sets=2, seed=0):
    """n_sets (x1, x2, lam, y) tuples resident in HBM; clips are circular
    shifts of a 64-clip synthetic bank (distinct per row)."""
    bank = torch.from_numpy(synth_bank(64, seed=20260227 + seed)).to(device)
    g = torch.Generator().manual_seed(seed)
    from acfe.frontend import sample_mixup_lambda
    from acfe.train import mix_labels

    sets = []
    for s in range(n_sets):
        xs, ys = [], []
        for _ in range(2):
            idx = torch.randint(0, 64, (batch,), generator=g)
            shift = torch.randint(0, N_SAMPLES, (batch,), generator=g)
            x = torch.empty((batch, N_SAMPLES), device=device)
            for i in range(batch):
                x[i] = torch.roll(bank[int(idx[i])], int(shift[i]))
            lab = torch.randint(0, classes, (batch,), generator=g)
            y = torch.zeros((batch, classes), device=device)
            y[torch.arange(batch), lab.to(device)] = 1
            xs.append(x)
            ys.append(y)
        torch.manual_seed(seed * 1000 + s)
        lam = sample_mixup_lambda(batch, 0.5, 0.25, device=device)
        sets.append((xs[0], xs[1], lam, mix_labels(ys[0], ys[1], lam)))
    return sets


def cpu_baseline(batch=2, steps=2, model="bird", classes=50):
    """Reference algorithm on the host (oracle/: numpy STFT + the reference's
    DENSE batch_dot mel, sequential PCEN scan, torch-CPU WRN fwd/bwd + Adam)."""
    from oracle import frontend as of
    from oracle import models as om
    from oracle.torch_ref import pcen_torch

    if model == "bird":
        from resnet.wr_resnet_bird import WRResNet
        fwd = om.wr_resnet_bird
    else:
        from resnet.wr_resnet import WRResNet
        fwd = om.wr_resnet
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    m = WRResNet(input_shape=(128, 513, 3), classes=classes, dropout=0.0)
    params = {k: v.detach().clone().requires_grad_("moving" not in k) for k, v in m.state_dict().items()}
    trainable = [v for k, v in params.items() if "moving" not in k]
    state = {k: v for k, v in params.items() if "moving" in k}
    mvec = [torch.zeros_like(p) for p in trainable]
    vvec = [torch.zeros_like(p) for p in trainable]
    w = of.mel_f(48000, 128, 100, 11000, 4096, 1000).astype(np.float32)
    raw = synth_bank(batch * 2, seed=777)
    lam = np.full(batch, 0.3)
    y = np.zeros((batch, classes), np.float32)
    y[np.arange(batch), np.arange(batch) % classes] = 1
    pc = torch.tensor([0.98, 2.0, 2.0, 0.04], dtype=torch.float32, requires_grad=True)

    def one_step(t):
        a, b = of.normalize(raw[:batch]), of.normalize(raw[batch:])
        x, _ = of.mix_up(a, y, b, y, lam)
        x = of.normalize(x).astype(np.float32)
        spec = np.abs(of.stft_pad_end(x, 4096, 281)).astype(np.float32) ** 2      # [B, T, F]
        mel = np.einsum("mf,btf->bmt", w, spec, optimize=True).astype(np.float32)   # dense mel (K5)
        feats = pcen_torch(torch.from_numpy(mel).transpose(1, 2).contiguous(), pc)  # [B, M, T]
        z = fwd(feats[:, None].repeat(1, 3, 1, 1).float(), params, True, state)
        loss = om.keras_loss(z, torch.from_numpy(y), "cce")
        loss.backward()
        with torch.no_grad():
            new, _, _ = om.keras_adam([p.detach() for p in trainable], [p.grad for p in trainable], mvec, vvec, t)
            for p, q in zip(trainable, new):
                p.copy_(q)
                p.grad = None

    one_step(1)
    t0 = time.perf_counter()
    for i in range(steps):
        one_step(i + 2)
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 4), "unit": "clips/s", "cores": cores, "kind": "port",
            "sample": f"{steps} timed training steps x {batch} clips (after 1 warm-up) of the CPU restatement: "
                      f"numpy STFT + dense mel batch_dot, sequential PCEN scan, torch-CPU {model} fwd/bwd "
                      f"(fp32, {cores} threads) + Keras Adam; {dt:.1f} s"}


def dominant_evidence(key: str, same_shape: bool):
    """(traffic, counters) of the dominant kernel of workload `key` (t1, wrn,
    t1_fp32, wrn_fp32, infer_fp32, stream_fp32, ...) from the committed PMC folds:
    profiles/pmc_dominant_<key>_<round>.json (HBM bytes per launch, FETCH_SIZE x2
    + WRITE_SIZE, tools/pmc_fold.py) and profiles/sq_dominant_<key>_<round>.json
    (SQ counters, tools/sq_json.py), newest round first; T1 also falls back to
    the earlier rounds' unsuffixed files.  Only used when this run has the
    measured launch shape (same_shape)."""
    if not same_shape:
        return None, None, None
    prof = ROOT / "profiles"

    def newest(kind):
        names = [f"{kind}_{key}_r{r:02d}.json" for r in range(9, 3, -1)]
        if key == "t1":
            names += [f"{kind}_r03.json", f"{kind}_r02b.json"]
        return next((prof / n for n in names if (prof / n).exists()), None)

    traffic = counters = src = None
    pmc = newest("pmc_dominant")
    if pmc is not None:
        try:
            d = json.loads(pmc.read_text())
            traffic = d.get("hbm_bytes_per_launch")
            # replayed from the committed PMC fold (rocprofv3 --pmc cannot run
            # inside this timed process): its file and the tree it measured
            src = {"file": f"profiles/{pmc.name}", "commit": d.get("commit"),
                   "over_algorithmic": d.get("traffic_over_algorithmic")}
        except ValueError:
            traffic = None
    sq = newest("sq_dominant")
    if sq is not None:
        try:
            d = json.loads(sq.read_text())
            counters = {k: d[k] for k in ("mfma_busy_per_simd", "wave_time_waiting", "valu_insts_per_mfma",
                                          "lds_bank_conflict_share")}
            counters["source"] = f"profiles/{sq.name}"
            counters["commit"] = d.get("commit")
        except (ValueError, KeyError):
            counters = None
    return traffic, src, counters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="clips per GPU")
    ap.add_argument("--classes", type=int, default=50)
    ap.add_argument("--model", choices=["bird", "wrn"], default="bird")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", dest="extra", action="store_false",
                    help="skip the secondary workloads (wr_resnet training, configs I and S) of the default run")
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--clips", type=int, default=4096, help="e2e: clips written to the TFRecord set")
    ap.add_argument("--no-cache", dest="cache", action="store_false",
                    help="e2e: stream every epoch from the shards (no HBM dataset cache)")
    ap.add_argument("--workload", choices=["train", "infer", "stream", "e2e"], default="train",
                    help="train = T1/T8 (the driver's line); infer = config I (B=256 fp32 wr_resnet fwd); "
                         "stream = config S (60-min recording, 3 s / 1.5 s windows, batch 1024)")
    a = ap.parse_args()
    if a.workload == "e2e":
        return run_e2e(a)
    if a.workload != "train":
        print(json.dumps(run_inference(a)), flush=True)
        return 0

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # `bench.py --gpus N` started directly: one process per GPU under
        # torch.distributed.run, started as a CHILD before anything here
        # touches the GPU; this process only relays its exit code.
        return launch_ranks(a.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks; measuring {world}",
              file=sys.stderr, flush=True)
    # ranks beyond the visible GPUs share them (the gloo rehearsal on one GPU)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import torch.distributed as dist

    if world > 1:
        backend = os.environ.get("ACFE_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    from acfe import ops

    ops.set_seed_rank(rank)  # per-replica dropout masks
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    out, _ = train_line(a.model, dtype, a.classes, a.batch, a.steps, a.warmup, rank, world, dev, dist)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_batch, a.cpu_steps, a.model, a.classes)
        # the other workloads' CPU rows (tools/cpu_baseline.py on a GPU box's
        # host cores, same host type), newest round first
        suite = next((p for p in (ROOT / "profiles" / f"r{r:02d}_cpu_baseline.json" for r in range(9, 1, -1))
                      if p.exists()), None)
        if suite is not None:
            try:
                out["cpu_baseline"]["suite"] = {"source": f"profiles/{suite.name}",
                                                **json.loads(suite.read_text())["rows"]}
            except (ValueError, KeyError):
                pass
    if rank == 0 and world == 1 and a.extra and a.model == "bird" and a.dtype == "bf16" and a.batch == 512:
        # the secondary workloads of BASELINE.json at reduced step counts, so
        # the driver's own run observes them: the metric's named model
        # (wr_resnet training, T1 shape), config I and config S
        torch.cuda.empty_cache()
        w, _ = train_line("wrn", torch.bfloat16, 2, 512, 5, 2, 0, 1, dev, dist)
        out["wrn"] = _summary(w)
        torch.cuda.empty_cache()
        out["infer"] = _summary(run_inference(a, workload="infer", steps=5, warmup=2, emit=False))
        torch.cuda.empty_cache()
        out["stream"] = _summary(run_inference(a, workload="stream", steps=2, warmup=1, emit=False))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def active_switches():
    """The ACFE_* environment switches of this process (A/B and diagnostic
    flags of acfe/ops.py and the C library; empty on the default product
    path) and the library that was loaded -- recorded in every bench line."""
    from acfe import _lib

    return {"env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("ACFE_")},
            "library": os.path.relpath(_lib.LIB_PATH, ROOT) if hasattr(_lib, "LIB_PATH") else None}


def _summary(o):
    """The fields of a secondary workload's line kept in the main line."""
    keep = ("metric", "value", "unit", "ms_per_step", "ms_per_step_median", "steps", "warmup", "dtype", "config",
            "roofline", "mel_pipeline", "model_tflops_fwd_bwd", "final_loss")
    r = {k: o[k] for k in keep if k in o}
    if "roofline" in r:
        r["roofline"] = {k: v for k, v in r["roofline"].items() if k != "kernel"}
    return r


def train_line(model_name, dtype, classes, batch, steps, warmup, rank, world, dev, dist):
    """Time `steps` training steps (after `warmup`) of model_name on HBM-resident
    synthetic batches; returns (the bench line without cpu_baseline, trainer)."""
    from acfe import ops
    from acfe.train import FrontEnd, Trainer

    if model_name == "bird":
        from resnet.wr_resnet_bird import WRResNet, flops_per_clip
    else:
        from resnet.wr_resnet import WRResNet
        flops_per_clip = None
    torch.manual_seed(1234 + rank)
    model = WRResNet(input_shape=(128, 513, 3), classes=classes, dtype=dtype).to(dev)
    if world > 1:  # replicas start from rank 0's weights
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, 0)
    frontend = FrontEnd(n_mels=128, dtype=dtype, device=dev).to(dev)
    trainer = Trainer(model, frontend, lr=0.01, loss="cce", device=dev)
    sets = make_batches(batch, classes, dev, n_sets=2, seed=rank)

    # dominant kernel: stage-1 block-0 3x3 conv (128 -> 128 ch at 128 x 256)
    target = model.blocks[0].conv21 if model_name == "bird" else model.blocks[1].conv2a
    K, R, S, C = target.weight.shape
    events: list = []
    mel_events: list = []

    def step(i):
        x1, x2, lam, y = sets[i % len(sets)]
        return trainer.step(x1, y, x2, lam)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    ops.watch_conv(target.weight, events)
    frontend.timer = mel_events
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step HIP events on the launch stream (no host sync inside the
    # timed region): the median step time is reported beside the mean
    sev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    sev[0].record()
    for i in range(steps):
        loss, _ = step(i)
        sev[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = [sev[i].elapsed_time(sev[i + 1]) for i in range(steps)]
    ops.watch_conv(target.weight, None)
    frontend.timer = None
    own = elapsed
    per_rank = [own]
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        per_rank = [float(g.item()) for g in gathered]
        elapsed = max(per_rank)
    loss_v = float(loss.item())
    if rank != 0:  # each rank's own line, on stderr (stdout carries rank 0's one JSON line)
        print(f"bench rank {rank}/{world}: {batch * steps / own:.1f} clips/s, {own / steps * 1e3:.3f} ms/step, "
              f"loss {loss_v:.5f}", file=sys.stderr, flush=True)

    def avg_ms(kind, evs):
        d = [e0.elapsed_time(e1) for k, e0, e1 in evs if k == kind]
        return float(np.mean(d)) if d else float("nan")

    fwd_ms, dgrad_ms, wgrad_ms = avg_ms("fwd", events), avg_ms("dgrad", events), avg_ms("wgrad", events)
    mel_ms = avg_ms("mel", mel_events)
    H_t = 128
    W_t = 256 if model_name == "bird" else 513
    flops_launch = 2.0 * batch * H_t * W_t * K * R * S * C
    peak = MI355X_PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else MI355X_PEAK_FP32_TFLOPS
    ach = flops_launch / (fwd_ms * 1e-3) / 1e12
    key = ("t1" if model_name == "bird" else "wrn") + ("" if dtype == torch.bfloat16 else "_fp32")
    traffic, tsrc, counters = dominant_evidence(key, batch == 512)
    clips = world * batch * steps
    value = clips / elapsed
    bird = model_name == "bird"
    out = {
        "metric": "clips/sec training (3s@48kHz, wr_resnet) at 1/2/4/8 GPU; mel pipeline GB/s",
        "value": round(value, 2),
        "unit": "clips/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "ms_per_step_median": round(float(np.median(step_ms)), 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic (SURVEY 8d chirps+noise, resident in HBM; random-init weights)",
        "config": {
            "workload": f"T1 training step: normalize/mix_up/STFT-mel/PCEN + {'wr_resnet_bird' if bird else 'wr_resnet'} fwd/bwd + Adam",
            "model": "wr_resnet_bird" if bird else "wr_resnet",
            "input": [128, 513, 3], "classes": classes, "global_batch": world * batch,
            "batch_per_gpu": batch, "seq_len": 513, "parallelism": f"dp{world}",
            "loss": "categorical_crossentropy", "optimizer": "adam(lr=0.01)",
        },
        "roofline": {
            "kernel": f"conv2d_fwd {R}x{S} {C}->{K} @ {H_t}x{W_t} " + (
                "(k_conv_fwd_g<float,128,BN>: fp32 implicit-im2col GEMM on v_mfma_f32_16x16x4f32, LDS-staged tiles)"
                if dtype != torch.bfloat16 else
                "(k_conv3x3_1w<1,2,true>: 4 rows x 64 px x 128 ch per workgroup of 4 waves, one per SIMD with 128 accumulators each, chunk-resident halo rows; 2x2 max-pool + dropout + BN sums of the previous tile between this tile's MFMA groups)"
                if bird else
                "(k_conv3x3_r64<4,1,true,true>: bn2a + ReLU applied while staging the input rows, dropout (+ keep bits) + BN sums of the previous tile between this tile's MFMA groups; persistent, 8 rows x 64 px x 64 ch per tile, 8 waves)"),
            "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": traffic, "traffic_source": tsrc,
            "avg_launch_ms": round(fwd_ms, 4), "flops_per_launch": flops_launch,
            "counters": counters,
            "dgrad_ms": round(dgrad_ms, 4), "wgrad_ms": round(wgrad_ms, 4),
            "dgrad_tflops": round(flops_launch / (dgrad_ms * 1e-3) / 1e12, 2),
            "wgrad_tflops": round(flops_launch / (wgrad_ms * 1e-3) / 1e12, 2),
        },
        "mel_pipeline": {
            "kernel": "k_mel_w4 (two waves per frame, packed-f32 complex arithmetic: frame+Hann+4096 rFFT+|X|^2+banded mel)",
            "avg_launch_ms": round(mel_ms, 4),
            "GBps": round(batch * FRONTEND_BYTES_PER_CLIP / (mel_ms * 1e-3) / 1e9, 2),
            "hbm_frac": round(batch * FRONTEND_BYTES_PER_CLIP / (mel_ms * 1e-3) / 1e9 / MI355X_PEAK_HBM_GBS, 4),
            "bytes_per_clip": FRONTEND_BYTES_PER_CLIP,
            # 68.87 MFLOP per clip (FFT + power + banded mel), fp32 VALU peak 157.3 TFLOP/s
            "valu_tflops": round(batch * 68.87e6 / (mel_ms * 1e-3) / 1e12, 2),
            "valu_frac": round(batch * 68.87e6 / (mel_ms * 1e-3) / 1e12 / 157.3, 4),
        },
        "per_rank_s": [round(v, 4) for v in per_rank],
        "grad_allreduce": ({"buckets": len(trainer.buckets.buckets), "bucket_bytes": 4 << 20,
                            "arena_bytes": trainer.arena.numel * 4, "overlapped_with_backward": True}
                           if trainer.buckets is not None else None),
        "model_tflops_fwd_bwd": round(3 * (flops_per_clip(model) if flops_per_clip else 64.956e9) * value / 1e12, 2),
        "final_loss": round(loss_v, 5),
        "switches": active_switches(),
    }
    return out, trainer


def launch_ranks(n: int) -> int:
    import socket
    import subprocess

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.run(cmd, env=env).returncode


def _write_shard(args):
    path, first, count, classes = args
    sys.path[:0] = [str(ROOT / "audio-training_amd")]
    import tfrecord as tfr

    bank = synth_bank(64, seed=20260227)
    rng = np.random.default_rng(first)
    with tfr.TFRecordWriter(path) as w:
        for i in range(first, first + count):
            raw = np.roll(bank[i % 64], int(rng.integers(0, N_SAMPLES)))
            lab = f"c{i % classes:02d}"
            w.write(tfr.audio_example(raw, f"r{i}", i, lab, lab))
    return count


def run_e2e(a):
    """T1 training fed END TO END from GZIP TFRecords (SURVEY 8d's "second run
    with the TFRecord loader"): `--clips` synthetic clips in the reference
    schema are written to 16 shards in a temp dir (not timed), then
    tfdataset.AudioDataset (reader threads: GZIP inflate + protobuf parse into
    pinned host batches, mix_up pairs) feeds acfe.train.Trainer.  value =
    clips/s of the timed steps, host loading included."""
    import tempfile
    from concurrent.futures import ProcessPoolExecutor

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    classes = a.classes
    labels = [f"c{i:02d}" for i in range(classes)]
    tmp = tempfile.mkdtemp(prefix="acfe_e2e_")
    nsh = 16
    per = -(-a.clips // nsh)
    jobs = [(os.path.join(tmp, f"{i:05d}.tfrecord"), i * per, min(per, a.clips - i * per), classes)
            for i in range(nsh) if a.clips - i * per > 0]
    t0 = time.perf_counter()
    print(f"e2e: writing {a.clips} clips into {len(jobs)} GZIP shards", file=sys.stderr, flush=True)
    with ProcessPoolExecutor(min(16, len(jobs))) as ex:
        for i, _ in enumerate(ex.map(_write_shard, jobs)):
            print(f"e2e: shard {i + 1}/{len(jobs)} written ({time.perf_counter() - t0:.1f} s)", file=sys.stderr,
                  flush=True)
    t_write = time.perf_counter() - t0
    import tfdataset
    from acfe.frontend import sample_mixup_lambda
    from acfe.train import FrontEnd, Trainer, mix_labels

    if a.model == "bird":
        from resnet.wr_resnet_bird import WRResNet
    else:
        from resnet.wr_resnet import WRResNet
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    torch.manual_seed(1234)
    model = WRResNet(input_shape=(128, 513, 3), classes=classes, dtype=dtype).to(dev)
    frontend = FrontEnd(n_mels=128, dtype=dtype, device=dev).to(dev)
    trainer = Trainer(model, frontend, lr=0.01, loss="cce", device=dev)
    ds = tfdataset.AudioDataset(tfdataset._files(tmp), labels, batch_size=a.batch, shuffle=True, augment=True,
                                device=dev, threads=16, drop_remainder=True, cache=a.cache)

    def step(batch):
        (x1, y1), (x2, y2) = batch
        lam = sample_mixup_lambda(x1.shape[0], 0.5, 0.25, device=dev)
        return trainer.step(x1, mix_labels(y1, y2, lam), x2, lam)[0]

    # epoch 1 streams from the shards (and, with --cache, fills the HBM cache):
    # timed on its own, the epoch count pass (get_dataset's) included
    t1 = time.perf_counter()
    n1 = 0
    for batch in ds:
        step(batch)
        n1 += 1
    torch.cuda.synchronize()
    first = time.perf_counter() - t1
    print(f"e2e: first epoch {n1} steps in {first:.1f} s ({n1 * a.batch / first:.0f} clips/s)", file=sys.stderr,
          flush=True)

    def epochs():
        while True:
            yield from ds

    it = epochs()
    t1 = time.perf_counter()
    for _ in range(a.warmup):
        step(next(it))
    torch.cuda.synchronize()
    print(f"e2e: {a.warmup} warm-up steps in {time.perf_counter() - t1:.1f} s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    n = 0
    for i in range(a.steps):
        loss = step(next(it))
        n += 1
        if (i + 1) % 10 == 0:
            print(f"e2e: {i + 1} timed steps, {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    import shutil

    shutil.rmtree(tmp, ignore_errors=True)
    out = {"metric": "clips/sec training end to end from GZIP TFRecords (3s@48kHz)", "value": round(n * a.batch / el, 2),
           "unit": "clips/s", "n_gpus": 1, "steps": n, "warmup": a.warmup,
           "ms_per_step": round(el / max(n, 1) * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
           "data": f"synthetic clips written as {len(jobs)} GZIP TFRecord shards ({a.clips} clips, {t_write:.1f} s to "
                   f"write, not timed), read by tfdataset.AudioDataset: 16 native reader threads (libdeflate "
                   f"inflate, each record decoded once), 4096-clip device shuffle pool, mix_up partners drawn "
                   f"from the pool; " + ("epochs after the first served from the HBM-resident dataset cache "
                                         "(dataset.cache()); " if a.cache else "every epoch streamed; ")
                   + f"host CPUs available to the process: {len(os.sched_getaffinity(0))}",
           "first_epoch": {"steps": n1, "s": round(first, 3), "clips_s": round(n1 * a.batch / first, 1)},
           "config": {"workload": "T1 end to end: TFRecord loader + training step",
                      "model": "wr_resnet_bird" if a.model == "bird" else "wr_resnet", "classes": classes,
                      "batch": a.batch}, "final_loss": round(float(loss.item()), 5)}
    print(json.dumps(out), flush=True)


def run_inference(a, workload=None, steps=None, warmup=None, emit=True):
    """Configs I and S of BASELINE.json (one GPU; shards over ranks with no
    collective, so only the single-GPU replica is measured here).  Returns the
    line.  `workload` given (the default run's secondary lines): the config's
    own settings, not the command line's.

    I: fused normalize/STFT/mel/PCEN + wr_resnet forward, batch 256, fp32.
    S: one 60-min 48 kHz recording resident in HBM, 3 s windows every 1.5 s
       read in place by the front-end kernel (centred STFT, constant padding as
       predict_utils.get_spect), PCEN per window batch, model forward, sigmoid;
       batch 1024 windows, fp32 (the reference default).  A step = the whole
       recording."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from acfe import ops
    from acfe.train import FrontEnd

    if workload is None:  # command line
        stream = a.workload == "stream"
        model_name = a.model if (stream or "--model" in sys.argv) else "wrn"
        dtype = torch.float32 if (a.dtype == "fp32" or ("--dtype" not in sys.argv and not stream)) else torch.bfloat16
        classes = a.classes if "--classes" in sys.argv else (2 if model_name == "wrn" else 50)
        bs_arg = a.batch if "--batch" in sys.argv else None
        steps, warmup = a.steps, a.warmup
    else:
        stream = workload == "stream"
        model_name = "bird" if stream else "wrn"
        dtype = torch.float32
        classes = 50 if stream else 2
        bs_arg = None
    if model_name == "bird":
        from resnet.wr_resnet_bird import WRResNet
    else:
        from resnet.wr_resnet import WRResNet
    torch.manual_seed(1234)
    model = WRResNet(input_shape=(128, 513, 3), classes=classes, dtype=dtype).to(dev).eval()
    frontend = FrontEnd(n_mels=128, dtype=dtype, device=dev).to(dev).eval()
    target = model.blocks[0].conv21 if model_name == "bird" else model.blocks[1].conv2a
    K, R, S, C = target.weight.shape
    events, mel_events = [], []
    if stream:
        sr, n, hop = 48000, 144000, 72000
        rec = torch.from_numpy(np.tile(synth_bank(8, seed=4242).reshape(-1), 1500)[: 60 * 60 * sr].copy()).to(dev)
        n_win = 1 + (rec.numel() - n) // hop
        bs = bs_arg or 1024

        @torch.no_grad()
        def step(i):
            outs = []
            for first in range(0, n_win, bs):
                cnt = min(bs, n_win - first)
                outs.append(ops.sigmoid(model(frontend.forward_windows(rec, first, cnt, n=n, hop=hop))))
            return outs
        units = n_win
    else:
        bs = bs_arg or 256
        x = make_batches(bs, classes, dev, n_sets=1)[0][0]

        @torch.no_grad()
        def step(i):
            return ops.sigmoid(model(frontend(x)))
        units = bs
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    ops.watch_conv(target.weight, events)
    frontend.timer = mel_events
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ops.watch_conv(target.weight, None)
    frontend.timer = None
    d = [e0.elapsed_time(e1) for k, e0, e1 in events if k == "fwd"]
    fwd_ms = float(np.mean(d)) if d else float("nan")
    dm = [e0.elapsed_time(e1) for k, e0, e1 in mel_events]
    mel_ms = float(np.mean(dm)) if dm else float("nan")
    H_t = 128
    W_t = 256 if model_name == "bird" else 513
    # one launch of the target conv covers at most bs clips
    n_launch = -(-units // bs)
    avg_clips = units / n_launch
    flops_launch = 2.0 * avg_clips * H_t * W_t * K * R * S * C
    peak = MI355X_PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else MI355X_PEAK_FP32_TFLOPS
    ach = flops_launch / (fwd_ms * 1e-3) / 1e12
    value = units * steps / elapsed
    key = ("stream" if stream else "infer") + ("_fp32" if dtype == torch.float32 else "_bf16")
    traffic, tsrc, counters = dominant_evidence(key, bs == (1024 if stream else 256))
    out = {
        "metric": ("windows/sec streaming inference (60-min 48 kHz recording, 3 s / 1.5 s windows)" if stream
                   else "clips/sec inference (3s@48kHz, front end + PCEN + wr_resnet fwd)"),
        "value": round(value, 2), "unit": "windows/s" if stream else "clips/s", "n_gpus": 1,
        "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic (SURVEY 8d chirps+noise, resident in HBM; random-init weights)",
        "config": {"workload": ("S: streaming predict, 2399 windows/recording, batch %d" % bs) if stream
                   else ("I: inference batch %d" % bs),
                   "model": "wr_resnet_bird" if model_name == "bird" else "wr_resnet", "classes": classes,
                   "units_per_step": units, "batch": bs},
        "roofline": {"kernel": f"conv2d_fwd {R}x{S} {C}->{K} @ {H_t}x{W_t}", "bound": "mfma",
                     "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                     "traffic": traffic, "traffic_source": tsrc, "avg_launch_ms": round(fwd_ms, 4),
                     "flops_per_launch": flops_launch, "counters": counters},
        "mel_pipeline": {"avg_launch_ms": round(mel_ms, 4),
                         "GBps": round(avg_clips * FRONTEND_BYTES_PER_CLIP / (mel_ms * 1e-3) / 1e9, 2)},
        "switches": active_switches(),
    }
    return out


if __name__ == "__main__":
    sys.exit(main() or 0)
