"""tfdataset.get_dataset / AudioDataset on the CPU device: the native reader
(acfe_tfr_* / acfe_example_audio), the pinned-chunk -> pool -> gather
pipeline, the shuffle-buffer epoch contract and the failure modes the
reference's tf.data pipeline tolerates (tfdataset.py:212-226, :297, :429-506,
:835-838):

* epoch_size / len(): the examples one epoch yields (labels kept, feature of
  the expected size), as get_a_dataset returns it (:853-857);
* one epoch = every kept example exactly once as a primary, labels attached
  to the right clip; mix_up partners are resident clips of the same dataset;
* a corrupt or truncated GZIP shard ends that file (the intact prefix is
  used), an unreadable file is skipped, NaN clips and unknown labels are
  dropped -- and nothing hangs;
* a consumer that stops early releases the reader threads (ADVICE r02
  medium #2).
"""
import gzip
import threading
import time

import numpy as np
import pytest
import torch

import tfrecord as tfr

N = 144000


def _clip(k):
    return np.full(N, 0.001 * k, np.float32)


def _write(path, ks, labels=("bird", "noise"), nan_at=()):
    with tfr.TFRecordWriter(path) as w:
        for k in ks:
            raw = _clip(k)
            if k in nan_at:
                raw[17] = np.nan
            lab = labels[k % len(labels)]
            w.write(tfr.audio_example(raw, f"r{k}", k, lab, lab))


def _ids(x):
    return [int(round(float(v) / 0.001)) for v in x[:, 0]]


@pytest.fixture()
def shards(tmp_path):
    d = tmp_path / "train"
    d.mkdir()
    _write(d / "00000.tfrecord", range(0, 23))
    _write(d / "00001.tfrecord", range(23, 40), labels=("bird", "noise", "other"))   # "other" dropped
    _write(d / "00002.tfrecord", range(40, 51), nan_at=(44,))                        # NaN clip dropped
    keep = [k for k in range(51) if not (23 <= k < 40 and k % 3 == 2) and k != 44]
    return d, keep


def _label_ok(k, y):
    lab = ("bird", "noise", "other")[k % 3] if 23 <= k < 40 else ("bird", "noise")[k % 2]
    return y[["bird", "noise"].index(lab)] == 1 and y.sum() == 1


@pytest.mark.parametrize("shuffle", [True, False])
def test_epoch_contract(shards, shuffle):
    import tfdataset

    d, keep = shards
    ds, remapped, epoch_size, labels, extra = tfdataset.get_dataset(
        d, ["bird", "noise"], batch_size=8, shuffle=shuffle, device="cpu", threads=3, shuffle_buffer=16)
    assert epoch_size == len(keep)
    assert len(ds) == -(-len(keep) // 8)
    for epoch in range(2):
        seen = []
        nb = 0
        for x, y in ds:
            assert x.shape[1:] == (N,) and y.shape[1] == 2
            for k, row in zip(_ids(x), y):
                assert _label_ok(k, row), k
            seen += _ids(x)
            nb += 1
        assert sorted(seen) == keep and nb == len(ds)


def test_pool_smaller_than_dataset_refills_slots(shards, monkeypatch):
    """A shuffle pool far smaller than the epoch (4-clip chunks, 6-clip
    buffer, 44 records): slots freed by each batch are refilled by the next
    chunks, so the stream neither stalls nor repeats or loses an example."""
    import tfdataset

    monkeypatch.setattr(tfdataset, "CHUNK_BYTES", 4 * 4 * N)
    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=3, device="cpu", threads=3,
                                shuffle_buffer=6, augment=True)
    assert ds.per_chunk == 4 and ds.pool_rows == 6 + 8
    t0 = time.perf_counter()
    seen = []
    for (x1, y1), (x2, y2) in ds:
        for k, row in zip(_ids(x1), y1):
            assert _label_ok(k, row)
        seen += _ids(x1)
    assert time.perf_counter() - t0 < 60
    assert sorted(seen) == keep


def test_mixup_pairs_and_drop_remainder(shards):
    import tfdataset

    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=8, augment=True, device="cpu",
                                threads=2, drop_remainder=True, shuffle_buffer=32)
    seen = []
    for (x1, y1), (x2, y2) in ds:
        assert x1.shape == x2.shape == (8, N)
        for k, row in zip(_ids(x2), y2):
            assert k in keep and _label_ok(k, row)
        seen += _ids(x1)
    assert len(seen) == (len(keep) // 8) * 8 and len(set(seen)) == len(seen)
    assert len(ds) == len(keep) // 8


def test_corrupt_truncated_and_unreadable_shards_do_not_hang(tmp_path):
    import tfdataset

    d = tmp_path / "train"
    d.mkdir()
    _write(d / "a.tfrecord", range(0, 6))
    _write(d / "b.tfrecord", range(6, 12))
    full = gzip.decompress((d / "b.tfrecord").read_bytes())
    # truncated GZIP stream (the file ends mid-deflate): records before the cut survive
    (d / "b.tfrecord").write_bytes(gzip.compress(full)[:-2000])
    _write(d / "c.tfrecord", range(12, 18))
    raw = bytearray(gzip.decompress((d / "c.tfrecord").read_bytes()))
    raw[len(raw) // 2] ^= 0xFF  # CRC failure in the middle record
    (d / "c.tfrecord").write_bytes(gzip.compress(bytes(raw)))
    (d / "d.tfrecord").write_bytes(b"not a gzip stream at all")
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=4, device="cpu", threads=4)
    t0 = time.perf_counter()
    got = sorted(k for x, _ in ds for k in _ids(x))
    assert time.perf_counter() - t0 < 60
    assert got[:6] == list(range(6))
    assert all(k < 18 for k in got) and len(got) == len(set(got))
    assert any(6 <= k < 12 for k in got) and any(12 <= k < 18 for k in got)
    assert len(got) == ds.count()


def test_early_stop_releases_threads(shards):
    import tfdataset

    d, _ = shards
    before = threading.active_count()
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=2, device="cpu", threads=3,
                                shuffle_buffer=2)
    for _ in range(3):
        it = iter(ds)
        next(it)
        it.close()  # a steps_per_epoch break / synced_batches stop
    deadline = time.time() + 10
    while threading.active_count() > before and time.time() < deadline:
        time.sleep(0.05)
    assert threading.active_count() <= before


def test_spectrogram_records(tmp_path):
    import tfdataset

    d = tmp_path / "train"
    d.mkdir()
    rng = np.random.default_rng(0)
    specs = []
    with tfr.TFRecordWriter(d / "s.tfrecord") as w:
        for k in range(3):
            s = rng.random((2049, 513), dtype=np.float32)
            specs.append(s)
            w.write(tfr.audio_example(_clip(k), f"r{k}", k, "bird", "bird", spectrogram=s))
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird"], batch_size=3, shuffle=False, device="cpu",
                                load_raw=False)
    (x, y), = list(ds)
    assert x.shape == (3, 2049, 513)
    for k in range(3):
        assert torch.equal(x[k], torch.from_numpy(specs[k]))


def test_mixup_partners_in_the_epoch_tail(tmp_path):
    """After the readers finish the pool drains; the last batches still draw
    mix_up partners from the last buffer-full of clips, not only from the
    batch's own primaries."""
    import tfdataset

    d = tmp_path / "train"
    d.mkdir()
    _write(d / "a.tfrecord", range(0, 40))
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=4, augment=True, device="cpu",
                                threads=1, shuffle_buffer=8, seed=3)
    batches = [(_ids(x1), _ids(x2)) for (x1, _), (x2, _) in ds]
    assert sorted(k for p, _ in batches for k in p) == list(range(40))
    outside = sum(1 for p, q in batches[-2:] for k in q if k not in p)
    assert outside > 0


@pytest.mark.gpu
def test_back_to_back_epochs_keep_gathered_clips(shards, cuda):
    """A consumer that breaks an epoch and starts the next one at once: the new
    epoch's first refills (side-stream copies into the pool) must wait for the
    previous epoch's gathers still queued on the compute stream (the pool's
    release event carries over epochs)."""
    import tfdataset

    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=8, device=cuda, threads=3,
                                shuffle_buffer=16)
    for _ in range(3):
        it = iter(ds)
        torch.cuda._sleep(1_000_000_000)  # the gathers of the batch below queue behind ~0.5 s of spinning
        x, y = next(it)
        it.close()
        it2 = iter(ds)
        x2, y2 = next(it2)
        it2.close()
        for xb, yb in ((x, y), (x2, y2)):
            for k, row in zip(_ids(xb.cpu()), yb.cpu()):
                assert k in keep and _label_ok(k, row), k


def test_dataset_cache_epochs(shards, monkeypatch):
    """cache=True (the reference's dataset.cache(), tfdataset.py:792-793): the
    first full epoch streams from the shards and keeps every clip resident;
    later epochs start no reader threads, still yield every kept example
    exactly once with its label, reshuffled, with mix_up partners from the
    resident clips; an epoch broken off early caches nothing."""
    import tfdataset

    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=8, device="cpu", threads=3,
                                shuffle_buffer=16, augment=True, cache=True)
    it = iter(ds)
    next(it)
    it.close()
    assert ds._cached is None  # broken off: not cached
    orders = []
    for epoch in range(3):
        if epoch == 2:  # cached epochs never touch the shards
            monkeypatch.setattr(tfdataset.AudioDataset, "_reader", lambda *a, **k: (_ for _ in ()).throw(
                AssertionError("reader started on a cached epoch")))
        seen = []
        for (x1, y1), (x2, y2) in ds:
            for k, row in zip(_ids(x1), y1):
                assert _label_ok(k, row), k
            for k, row in zip(_ids(x2), y2):
                assert k in keep and _label_ok(k, row), k
            seen += _ids(x1)
        assert sorted(seen) == keep
        orders.append(seen)
        assert ds._cached is not None
    assert orders[1] != orders[2]  # reshuffled every epoch


def test_dataset_cache_over_budget_streams(shards):
    import tfdataset

    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=8, device="cpu", threads=3,
                                shuffle_buffer=16, cache=True, cache_bytes=4 * N * 10)
    for _ in range(2):
        assert sorted(k for x, _ in ds for k in _ids(x)) == keep
    assert ds._cached is None and not ds.cache


def test_dataset_cache_with_short_epoch_size_does_not_hang(shards, monkeypatch):
    """cache=True with a caller epoch_size below the true record count (ADVICE
    r04 medium): the pool is planned for too few clips, so the caching epoch
    runs out of slots; it must fall back to streaming (every kept example once,
    nothing cached) instead of waiting for slot releases that never come."""
    import tfdataset

    monkeypatch.setattr(tfdataset, "CHUNK_BYTES", 4 * 4 * N)
    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=3, device="cpu", threads=3,
                                shuffle_buffer=6, augment=True, cache=True, epoch_size=5)
    for _ in range(2):
        t0 = time.perf_counter()
        seen = []
        for (x1, y1), _ in ds:
            for k, row in zip(_ids(x1), y1):
                assert _label_ok(k, row), k
            seen += _ids(x1)
        assert time.perf_counter() - t0 < 60
        assert sorted(seen) == keep
        assert ds._cached is None


@pytest.mark.gpu
def test_dataset_cache_on_device(shards, cuda):
    """The HBM-resident cache on the GPU: epochs 2-3 gather every kept clip
    (with its label) from the device pool the first epoch filled."""
    import tfdataset

    d, keep = shards
    ds = tfdataset.AudioDataset(tfdataset._files(d), ["bird", "noise"], batch_size=8, device=cuda, threads=3,
                                shuffle_buffer=16, augment=True, cache=True)
    for epoch in range(3):
        seen = []
        for (x1, y1), (x2, y2) in ds:
            for k, row in zip(_ids(x1.cpu()), y1.cpu()):
                assert _label_ok(k, row), k
            for k, row in zip(_ids(x2.cpu()), y2.cpu()):
                assert k in keep and _label_ok(k, row), k
            seen += _ids(x1.cpu())
        assert sorted(seen) == keep
        assert ds._cached is not None
