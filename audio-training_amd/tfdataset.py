"""Input pipeline of the acfe path (reference tfdataset.py:193-506, :983-1228).

get_dataset(dir, labels, global_epoch=None, **args) keeps the reference
signature and return tuple (dataset, remapped, epoch_size, labels,
extra_label_map).  The dataset hands out DEVICE batches: x [B, 144000] fp32 raw
audio (normalize / mix_up / STFT / mel run on the GPU, acfe.train.FrontEnd), or
[B, 2049, 513] stored magnitude spectrograms (load_raw=False), and y
[B, len(labels)] one-hot; with augment=True each item is a pair of batches for
mix_up (tfdataset.py:473-481).

Pipeline (every record is inflated and parsed ONCE):

  reader threads   native shard reader (tfrecord.ShardReader: libdeflate
                   inflate, hardware CRC-32C) + acfe_example_audio, which
                   copies the record's floats straight into a slot of a
                   pinned staging chunk (no per-clip Python copies; ctypes
                   drops the GIL inside both calls)
  mover thread     one host->device copy per full chunk (64 clips) on a side
                   stream, its clips scattered into free slots of the
                   device-resident clip pool (acfe_copy_rows)
  consumer         the pool is the shuffle buffer (tfdataset.py:835-838,
                   4096 examples): a batch is B slots drawn uniformly from the
                   resident clips and gathered on the device (acfe_copy_rows),
                   their slots refilled as the next chunks arrive; each
                   example is a primary exactly once per epoch (one pass, as
                   the reference's dataset)

cache=True (the reference's dataset.cache(), "Caching to mem",
tfdataset.py:792-793, 832-834): the decoded clips are kept in HBM.  The first
epoch streams as above into a pool sized for the whole epoch whose slots are
never recycled; once it has run to its end, later epochs start no reader
threads at all -- the same shuffle buffer is fed from the resident clips in
their decode order, so an epoch costs device gathers only (288 GB of HBM hold
~250 000 decoded 3 s clips; the default budget is half of the device's
memory, beyond it the dataset streams every epoch).  The reference turns its
cache off for mix_up training (tfdataset.py:469-470) because its partners come
from a second, independently shuffled pipeline; here partners are drawn from
the resident pool, so the cache applies to mix_up training as well.

mix_up partners.  The reference zips a second, independently shuffled full
pass over the same records (tfdataset.py:473-480), i.e. it decodes every
record twice to pair each example with a random other example.  Here the
partner batch is B clips drawn uniformly from the same resident pool (the
primaries of the current batch included, as an independent pass may also
return them) and gathered on the device: the same distribution of pairs
(uniform over the dataset, up to the shuffle-buffer locality both pipelines
have), without the second decode.  In the epoch's tail, once the readers are
done and the pool drains, the clips of the last buffer-full of primaries stay
in the partner pool (nothing overwrites a released slot any more), so the last
batches are not paired mostly with themselves.
"""
from __future__ import annotations

import ctypes
import logging
import queue
import random
import threading
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np
import torch

import tfrecord as tfr

N_SAMPLES = 48000 * 3
HOP_LENGTH, NFFT, SR, BREAK_FREQ, FMIN, FMAX = 281, 4096, 48000, 1000, 100, 11000  # tfdataset.py:42-56
N_MELS = 160
DIMENSIONS = (160, 513, 1)
SPEC_SHAPE = (2049, 513)
SHUFFLE_BUFFER = 4096          # ds.shuffle(4096) per dataset, tfdataset.py:835-838
CHUNK_BYTES = 64 << 20         # pinned staging chunk (64 raw clips)
POOL_BYTES = 6 << 30           # cap of the device-resident shuffle pool
_POLL = 0.1                    # seconds between stop-flag checks of blocked threads
_TEXT_CAP = 256


def _lib():
    from acfe._lib import lib

    return lib


class _Stop(Exception):
    pass


class _Staging:
    """Pinned host chunks of `per` slots that reader threads fill concurrently.
    claim() hands out (chunk, slot) positions of the chunk being filled;
    commit() records the slot's label (-1 = filtered out after the copy); a
    chunk whose positions are all handed out and committed goes to `full`."""

    def __init__(self, buf, stop):
        nchunks, per = buf.shape[0], buf.shape[1]
        self.per, self.stop = per, stop
        self.buf = buf
        self.free: queue.Queue = queue.Queue()
        for c in range(nchunks):
            self.free.put(c)
        self.full: queue.Queue = queue.Queue()
        self.lock = threading.Lock()
        self.cur = None
        self.pos = 0
        self.pending = [0] * nchunks
        self.sealed = [False] * nchunks
        self.count = [0] * nchunks
        self.labels = np.full((nchunks, per), -1, np.int32)

    def claim(self):
        while True:
            with self.lock:
                if self.cur is not None:
                    c, p = self.cur, self.pos
                    self.pos += 1
                    self.pending[c] += 1
                    if self.pos == self.per:
                        self._seal(c, self.per)
                    return c, p
            try:  # wait for a free chunk without holding the lock
                c = self.free.get(timeout=_POLL)
            except queue.Empty:
                if self.stop.is_set():
                    raise _Stop
                continue
            with self.lock:
                if self.cur is None:
                    self.cur, self.pos = c, 0
                    self.labels[c].fill(-1)
                    self.sealed[c] = False
                else:  # another thread opened one meanwhile
                    self.free.put(c)

    def _seal(self, c, n):  # lock held
        self.cur = None
        self.sealed[c] = True
        self.count[c] = n
        if self.pending[c] == 0:
            self.full.put(c)

    def commit(self, c, p, label):
        with self.lock:
            self.labels[c, p] = label
            self.pending[c] -= 1
            if self.sealed[c] and self.pending[c] == 0:
                self.full.put(c)

    def flush(self):
        """All readers are done: seal the partially filled chunk."""
        with self.lock:
            if self.cur is not None:
                c, n = self.cur, self.pos
                if n == 0:
                    self.cur = None
                    self.free.put(c)
                else:
                    self._seal(c, n)


class AudioDataset:
    """Iterable over device batches; one pass = one epoch."""

    def __init__(self, files, labels, batch_size=32, shuffle=True, augment=False, device=None, threads=8,
                 drop_remainder=False, seed=0, label_map=None, record_shard=None, load_raw=True,
                 shuffle_buffer=SHUFFLE_BUFFER, epoch_size=None, cache=False, cache_bytes=None):
        """record_shard=(rank, world): keep only the records whose (file index
        + record index) % world == rank -- data-parallel sharding when there
        are fewer shard files than ranks (otherwise ranks take whole files).
        load_raw=False: batches of the stored magnitude spectrograms
        [B, 2049, 513] (audio/spectogram, tfdataset.py:1032-1034, 1081-1082);
        there is no mix_up on that path (tfdataset.py:503-504).
        cache: keep the decoded clips device-resident after the first full
        epoch (module docstring); cache_bytes caps the device memory it may
        take (default: half of the device's memory)."""
        self.files, self.labels = list(files), list(labels)
        self.record_shard = record_shard
        self.load_raw = load_raw
        if not load_raw:
            augment = False
        self.batch_size, self.shuffle, self.augment = int(batch_size), shuffle, augment
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.threads, self.drop_remainder, self.seed = max(1, int(threads)), drop_remainder, seed
        self.label_index = {l: i for i, l in enumerate(self.labels)}
        self.label_map = label_map or {}
        self.epoch = 0
        self.key = b"audio/raw" if load_raw else b"audio/spectogram"
        self.shape = (N_SAMPLES,) if load_raw else SPEC_SHAPE
        self.nfloats = int(np.prod(self.shape))
        clip_bytes = 4 * self.nfloats
        self.per_chunk = max(1, min(64, CHUNK_BYTES // clip_bytes))
        buf = max(shuffle_buffer if shuffle else 0, self.batch_size)
        buf = min(buf, max(self.batch_size, POOL_BYTES // clip_bytes))
        self.buffer = buf
        self.pool_rows = buf + 2 * self.per_chunk
        self._epoch_size = epoch_size
        self._pool = None
        self._dstage = None
        self._stage_buf = None
        self._last_ev = None  # event after the newest gathers from the pool (orders the next epoch's refills)
        self.error = None
        self.cache = bool(cache)
        self.cache_bytes = cache_bytes
        self._cached = None  # (pool rows in decode order, slot labels) once a whole epoch is resident

    # ---------------------------------------------------------------- counting
    def _label_of(self, text: str):
        lab = self.label_map.get(text, text)
        return self.label_index.get(lab)

    def _keep(self, i, r):
        shard = self.record_shard
        return shard is None or (i + r) % shard[1] == shard[0]

    def _count_file(self, i, path):
        lib = _lib()
        text = ctypes.create_string_buffer(_TEXT_CAP)
        cnt = ctypes.c_int64()
        scratch = np.empty(self.nfloats, np.float32)  # the NaN / Inf filter needs the values
        n = 0
        try:
            with tfr.ShardReader(path) as rd:
                r = 0
                while True:
                    try:
                        rec = rd.next()
                    except IOError:
                        break
                    if rec is None:
                        break
                    if self._keep(i, r):
                        fl = lib.acfe_example_audio(rec[0], rec[1], self.key, scratch.ctypes.data, self.nfloats,
                                                    text, _TEXT_CAP, ctypes.byref(cnt))
                        if fl >= 0 and fl & 2 and self._label_of(text.value.decode(errors="replace")) is not None:
                            n += 1
                    r += 1
        except IOError as e:
            logging.warning("skipping unreadable shard %s: %s", path, e)
        return n

    def count(self) -> int:
        """Examples one epoch yields (the reference's epoch_size, computed by
        its get_distribution pass over the dataset, tfdataset.py:853-857):
        records of this rank's share whose label is kept and whose float
        feature has the expected size and is finite (the filters of
        read_tfrecord / filter_nan_samples, tfdataset.py:297)."""
        if self._epoch_size is None:
            stable = {f: i for i, f in enumerate(self.files)}
            with ThreadPoolExecutor(min(self.threads, max(1, len(self.files)))) as ex:
                self._epoch_size = sum(ex.map(lambda f: self._count_file(stable[f], f), self.files))
        return self._epoch_size

    def __len__(self):
        n = self.count()
        b = self.batch_size
        return n // b if self.drop_remainder else -(-n // b)

    # ---------------------------------------------------------------- readers
    def _reader(self, files, stage: _Staging, stop, stable):
        lib = _lib()
        text = ctypes.create_string_buffer(_TEXT_CAP)
        cnt = ctypes.c_int64()
        row = stage.buf[0, 0].numel()
        base = stage.buf.data_ptr()
        while not stop.is_set():
            try:
                path = files.get_nowait()
            except queue.Empty:
                return
            i = stable.get(path, 0)
            try:
                with tfr.ShardReader(path) as rd:
                    r = -1
                    while not stop.is_set():
                        r += 1
                        try:
                            rec = rd.next()
                        except IOError:  # corrupt record: the rest of the file is dropped (tfdataset.py:226)
                            logging.warning("corrupt record %d in %s: rest of the file skipped", r, path)
                            break
                        if rec is None:
                            break
                        if not self._keep(i, r):
                            continue
                        fl = lib.acfe_example_audio(rec[0], rec[1], self.key, None, self.nfloats, text, _TEXT_CAP,
                                                    ctypes.byref(cnt))
                        if fl < 0 or not fl & 1 or cnt.value != self.nfloats:
                            continue
                        lab = self._label_of(text.value.decode(errors="replace"))
                        if lab is None:
                            continue
                        c, p = stage.claim()
                        kept = -1  # NaN / Inf filter (tfdataset.py:297): the slot stays empty
                        try:
                            dst = base + ((c * stage.per + p) * row) * 4
                            fl = lib.acfe_example_audio(rec[0], rec[1], self.key, dst, self.nfloats, None, 0,
                                                        ctypes.byref(cnt))
                            if fl >= 0 and fl & 2:
                                kept = lab
                        finally:  # a claimed slot is always committed, or its chunk never fills
                            stage.commit(c, p, kept)
            except _Stop:
                return
            except Exception as e:  # noqa: BLE001 -- an unreadable shard ends that file, not the epoch
                logging.warning("skipping shard %s: %s", path, e)

    # ---------------------------------------------------------------- pool
    def _cache_plan(self) -> bool:
        """Can the whole epoch be kept resident?  If so the pool is sized for it."""
        if not self.cache:
            return False
        n = self.count()
        budget = self.cache_bytes
        if budget is None:
            if self.device.type == "cuda":
                # what is free now, less a quarter of the device for the
                # activations / workspaces the training step has yet to take
                free, total = torch.cuda.mem_get_info(self.device)
                budget = max(0, min(total // 2, free - total // 4))
            else:
                budget = 1 << 30
            logging.info("dataset cache budget %.1f GB", budget / 1e9)
        need = (n + self.per_chunk) * 4 * self.nfloats
        if need > budget:
            logging.warning("dataset cache: %d clips need %.1f GB > budget %.1f GB; streaming every epoch", n,
                            need / 1e9, budget / 1e9)
            self.cache = False
            return False
        rows = max(self.pool_rows, n + self.per_chunk)
        if self._pool is not None and self._pool.shape[0] < rows:
            self._pool = None
        self.pool_rows = rows
        return True

    def _ensure_pool(self):
        if self._pool is None:
            self._pool = torch.empty((self.pool_rows, self.nfloats), dtype=torch.float32, device=self.device)
            if self.device.type == "cuda":  # one chunk on the device: pinned -> here -> scattered into free slots
                self._dstage = torch.empty((self.per_chunk, self.nfloats), dtype=torch.float32, device=self.device)
        return self._pool

    def _copy_rows(self, src, src_idx, dst, dst_idx, n):
        """dst[dst_idx[i]] = src[src_idx[i]] on the device (acfe_copy_rows; the
        index lists are host ints, copied to the device on the current stream)."""
        from acfe._lib import call
        from acfe._torch import stream

        def dev_idx(ix, rows):
            if ix is None:
                return None
            a = np.asarray(ix, np.int32)
            assert a.min() >= 0 and a.max() < rows
            return torch.from_numpy(a).pin_memory().to(self.device, non_blocking=True)

        si, di = dev_idx(src_idx, src.shape[0]), dev_idx(dst_idx, dst.shape[0])
        call("acfe_copy_rows", src.data_ptr(), self.nfloats, src.shape[0], None if si is None else si.data_ptr(),
             dst.data_ptr(), self.nfloats, dst.shape[0], None if di is None else di.data_ptr(), n, self.nfloats,
             stream())
        return si, di  # (kept alive by the caller until the launch's stream has passed them)

    def _mover(self, stage: _Staging, ready: queue.Queue, slots: "_SlotPool", stop, readers_done):
        """Full pinned chunks -> the device pool: one host->device copy per
        chunk into a device staging chunk, then its valid rows are scattered
        into free pool slots (acfe_copy_rows) once the batch gathers that last
        read those slots have run (event of their release)."""
        try:
            cuda = self.device.type == "cuda"
            cs = torch.cuda.Stream(self.device) if cuda else None
            pool = self._pool
            while True:
                try:
                    c = stage.full.get(timeout=_POLL)
                except queue.Empty:
                    if stop.is_set():
                        return
                    if readers_done.is_set() and stage.full.empty():
                        with stage.lock:
                            idle = stage.cur is None and not any(stage.pending)
                        if idle:
                            ready.put(None)
                            return
                    continue
                n = stage.count[c]
                labels = stage.labels[c, :n]
                valid = [j for j in range(n) if labels[j] >= 0]
                if not valid:
                    stage.free.put(c)
                    continue
                got = slots.acquire(len(valid), stop)
                if got is None:
                    return
                dst, ev = got
                if cuda:
                    with torch.cuda.stream(cs):
                        if ev is not None:
                            cs.wait_event(ev)
                        self._dstage[:n].copy_(stage.buf[c, :n], non_blocking=True)
                        keep = self._copy_rows(self._dstage, valid, pool, dst, len(valid))
                        done = torch.cuda.Event()
                        done.record(cs)
                    done.synchronize()
                    del keep
                else:
                    pool.index_copy_(0, torch.tensor(dst, dtype=torch.int64),
                                     stage.buf[c, torch.tensor(valid, dtype=torch.int64)])
                out_labels = labels[valid].copy()
                stage.free.put(c)
                ready.put((dst, out_labels))
        except Exception as e:  # noqa: BLE001
            self.error = e
            logging.exception("loader mover thread failed")
            ready.put(None)

    def _draw(self, rng, live, used, target, done, augment):
        """One batch from the shuffle buffer `live` (uniform draw without
        replacement) and its mix_up partners -> (pick, partner)."""
        b = min(self.batch_size, len(live))
        if self.shuffle:
            pick = []
            for _ in range(b):  # uniform draw without replacement (swap-remove)
                j = rng.randrange(len(live))
                live[j], live[-1] = live[-1], live[j]
                pick.append(live.pop())
        else:
            pick = live[:b]
            del live[:b]
        partner = None
        if augment:
            # mix_up partners: any resident clip.  Once the readers are done
            # (nothing refills a released slot any more) the clips of the last
            # `target` primaries stay valid partners too, so the tail batches
            # do not shrink to pairing the batch with itself (the reference
            # draws partners from an independent second pass, tfdataset.py:473-480)
            resident = live + pick + (used[-target:] if done else [])
            partner = [resident[rng.randrange(len(resident))] for _ in range(b)]
        used.extend(pick)
        if len(used) > 2 * target:
            del used[:-target]
        return pick, partner

    def _stream_cached(self, augment, rng):
        """An epoch over the device-resident clips: the shuffle buffer is fed
        from the cache in decode order (no reader threads, no host copies)."""
        order, lab = self._cached
        slots = _SlotPool(0)  # nothing is ever refilled: releases are no-ops
        slots.keep = True
        target = self.buffer if self.shuffle else self.batch_size
        live: list[int] = []
        used: list[int] = []
        pos = 0
        while True:
            while pos < len(order) and len(live) < target:
                live.append(order[pos])
                pos += 1
            done = pos == len(order)
            if len(live) < self.batch_size and (not live or self.drop_remainder):
                return
            pick, partner = self._draw(rng, live, used, target, done, augment)
            yield pick, partner, lab, slots

    def _stream(self, augment):
        """Generator of (primary slots, partner slots or None, slot labels,
        slot pool) per batch of one epoch."""
        rng = random.Random(self.seed + 1000003 * self.epoch)
        if self._cached is not None:
            yield from self._stream_cached(augment, rng)
            return
        caching = self._cache_plan()
        files = list(self.files)
        if self.shuffle:
            rng.shuffle(files)  # load_dataset shuffles the file names (tfdataset.py:195-197)
        stable = {f: i for i, f in enumerate(self.files)}
        stop, readers_done = threading.Event(), threading.Event()
        if self._stage_buf is None:  # pinned once per dataset, reused every epoch
            self._stage_buf = torch.empty((max(4, self.threads // 2), self.per_chunk, self.nfloats),
                                          dtype=torch.float32, pin_memory=self.device.type == "cuda")
        stage = _Staging(self._stage_buf, stop)
        self.error = None
        self._ensure_pool()
        fq: queue.Queue = queue.Queue()
        for f in files:
            fq.put(f)
        # the previous epoch's last gathers may still be queued on the compute
        # stream: the first refill of this epoch waits for their event
        slots = _SlotPool(self.pool_rows, self._last_ev)
        slots.keep = caching  # caching epoch: every clip keeps its slot
        order: list[int] = []  # caching: slots in decode order
        ready: queue.Queue = queue.Queue()
        nthreads = min(self.threads, max(1, len(files)))
        readers = [threading.Thread(target=self._reader, args=(fq, stage, stop, stable), daemon=True)
                   for _ in range(nthreads)]
        for t in readers:
            t.start()

        def watch():
            for t in readers:
                t.join()
            stage.flush()
            readers_done.set()

        watcher = threading.Thread(target=watch, daemon=True)
        watcher.start()
        mover = threading.Thread(target=self._mover, args=(stage, ready, slots, stop, readers_done), daemon=True)
        mover.start()
        live: list[int] = []                   # resident slots not yet used as a primary this epoch
        used: list[int] = []                   # slots already used as a primary (mix_up partners in the tail)
        lab = np.full(self.pool_rows, -1, np.int32)
        # the shuffle buffer: batches are drawn once `target` clips are resident
        # (or the epoch's records are exhausted); the pool holds target + 2
        # chunks, so the mover always finds free slots while the buffer refills
        target = self.buffer if self.shuffle else self.batch_size
        done = False
        try:
            while True:
                while not done and len(live) < target:
                    item = ready.get()
                    if item is None:
                        done = True
                        break
                    dst, labels = item
                    lab[dst] = labels
                    live.extend(dst)
                    if caching:
                        order.extend(dst)
                if self.error is not None:
                    raise RuntimeError("TFRecord loader failed") from self.error
                if len(live) < self.batch_size:  # the stream has ended (the fill loop stops only then)
                    if not live or self.drop_remainder:
                        break
                pick, partner = self._draw(rng, live, used, target, done, augment)
                yield pick, partner, lab, slots
            if caching and done and self.error is None and slots.keep:
                # the whole epoch went through: later epochs run from the device
                self._cached = (order, lab.copy())
        finally:
            stop.set()
            for t in readers + [watcher, mover]:
                t.join(timeout=5)

    def _labels(self, rows, lab):
        """One-hot labels, copied to the device asynchronously from pinned
        memory (a pageable source would make the copy wait for the queue)."""
        cuda = self.device.type == "cuda"
        y = torch.zeros((len(rows), len(self.labels)), dtype=torch.float32, pin_memory=cuda)
        y[torch.arange(len(rows)), torch.from_numpy(lab[np.asarray(rows)].astype(np.int64))] = 1.0
        return y.to(self.device, non_blocking=True)

    def _gather(self, rows):
        pool = self._pool
        b = len(rows)
        if self.device.type != "cuda":
            return pool.index_select(0, torch.tensor(rows, dtype=torch.int64)).reshape((b,) + self.shape)
        out = torch.empty((b,) + self.shape, dtype=torch.float32, device=self.device)
        self._copy_rows(pool, rows, out.view(b, self.nfloats), None, b)
        return out

    def __iter__(self):
        augment = self.augment
        self.epoch += 1
        n = 0
        for pick, partner, lab, slots in self._stream(augment):
            x1 = self._gather(pick)
            y1 = self._labels(pick, lab)
            if augment:
                x2 = self._gather(partner)
                y2 = self._labels(partner, lab)
            # the primaries' slots are free for new clips once the gathers
            # above have run (an event on the launch stream orders the refill)
            ev = None
            if self.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
            slots.release(pick, ev)
            if ev is not None:
                self._last_ev = ev
            n += len(pick)
            yield ((x1, y1), (x2, y2)) if augment else (x1, y1)
        if self._epoch_size is None and self.record_shard is None:
            self._epoch_size = n


class _SlotPool:
    """Free slots of the device clip pool.  release() returns a batch's
    primary slots with the event recorded after the gathers that read them;
    acquire(n) hands out n free slots and the newest such event (events of
    one stream complete in order, so waiting for it covers every older one)."""

    def __init__(self, rows, ev=None):
        self.free = list(range(rows - 1, -1, -1))
        self.ev = ev
        self.keep = False  # dataset cache: released slots keep their clips
        self.held: list[int] = []  # slots released while keeping (given back if the cache is abandoned)
        self.cv = threading.Condition()

    def release(self, rows, ev):
        with self.cv:
            (self.held if self.keep else self.free).extend(rows)
            if ev is not None:
                self.ev = ev
            self.cv.notify_all()

    def acquire(self, n, stop):
        with self.cv:
            if self.keep and len(self.free) < n:
                # the epoch holds more clips than the pool was sized for (a
                # caller's epoch_size below the true record count): stop
                # caching rather than wait for releases that never come back
                logging.warning("dataset cache: more clips than planned; this epoch streams, nothing is cached")
                self.keep = False
                self.free.extend(self.held)
                self.held = []
            while len(self.free) < n:
                if stop.is_set():
                    return None
                self.cv.wait(timeout=_POLL)
            out = [self.free.pop() for _ in range(n)]
            return out, self.ev


def _files(dir):
    d = Path(dir)
    files = sorted(d.glob("*.tfrecord")) or sorted(d.rglob("*.tfrecord"))
    return [str(f) for f in files]


def count_examples(dir) -> int:
    n = 0
    for f in _files(dir):
        with tfr.ShardReader(f) as rd:
            while True:
                try:
                    if rd.next() is None:
                        break
                except IOError:
                    break
                n += 1
    return n


def get_dataset(dir, labels, global_epoch=None, **args):
    """tfdataset.get_dataset (tfdataset.py:429-506) -> (dataset, remapped,
    epoch_size, labels, extra_label_map).  epoch_size is the number of
    examples one epoch yields (the reference counts them with a full pass,
    get_distribution, :853-857; so does this: AudioDataset.count inflates every
    shard and checks every record's label and float list -- a full decode
    pass at startup -- unless args["epoch_size"] gives the number).  Extra keys
    accepted here: device, threads, seed, label_map, record_shard, files,
    drop_remainder, shuffle_buffer, cache_bytes; cache (the reference's
    dataset.cache(), off unless asked for) keeps the decoded clips in HBM."""
    global N_MELS, FMIN, FMAX, NFFT, BREAK_FREQ
    if args.get("n_mels"):
        N_MELS = args["n_mels"]
    if args.get("fmin") is not None:
        FMIN, FMAX = args.get("fmin", FMIN), args.get("fmax", FMAX)
    if args.get("n_fft") is not None:
        NFFT = args["n_fft"]
    if args.get("break_freq") is not None:
        BREAK_FREQ = args["break_freq"]
    files = args.get("files") or _files(dir)
    if not files:
        raise FileNotFoundError(f"no *.tfrecord under {dir}")
    labels = list(labels)
    remapped = {l: [l] for l in labels}
    load_raw = args.get("load_raw", True)
    ds = AudioDataset(files, labels, batch_size=args.get("batch_size") or 32, shuffle=args.get("shuffle", True),
                      augment=args.get("augment", False) and load_raw, device=args.get("device"),
                      threads=args.get("threads", 8), seed=args.get("seed", 0),
                      drop_remainder=args.get("drop_remainder", False), label_map=args.get("label_map"),
                      record_shard=args.get("record_shard"), load_raw=load_raw,
                      shuffle_buffer=args.get("shuffle_buffer", SHUFFLE_BUFFER), epoch_size=args.get("epoch_size"),
                      cache=args.get("cache", False), cache_bytes=args.get("cache_bytes"))
    epoch_size = ds.count()
    logging.info("dataset %s: %d shards, %d labels, %d examples", dir, len(files), len(labels), epoch_size)
    return ds, remapped, epoch_size, labels, {}
