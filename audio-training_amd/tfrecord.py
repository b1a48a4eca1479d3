"""GZIP TFRecord files of tf.train.Example protos, without TensorFlow.

On-disk contract of the reference (audiowriter.py:67-174, :259-277 writes it;
tfdataset.py:212-226, :983-1060 reads it):
  record  = uint64 len (LE) | uint32 masked_crc32c(len bytes) | data | uint32 masked_crc32c(data)
  masked  = ((crc >> 15) | (crc << 17)) + 0xa282ead8   (mod 2**32)
  data    = tf.train.Example { Features features = 1 { map<string, Feature> feature = 1 } }
  Feature = oneof { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3 }
The protobuf wire format is written/parsed by hand (varints, length-delimited
fields, packed floats/int64s); CRC-32C comes from libacfe (host C code).
"""
from __future__ import annotations

import ctypes
import gzip
import struct
from typing import Iterable, Iterator

import numpy as np

_MASK_DELTA = 0xA282EAD8


def _crc32c(b: bytes) -> int:
    from acfe._lib import lib

    return lib.acfe_crc32c(b, len(b), 0)


def masked_crc(b: bytes) -> int:
    c = _crc32c(b)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


# ------------------------------------------------------------------ protobuf wire format
def _varint(n: int) -> bytes:
    if n < 0:
        n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos: int) -> tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _feature(value) -> bytes:
    """value: bytes/str/list[bytes] -> BytesList; float ndarray/list -> FloatList; int -> Int64List."""
    if isinstance(value, (bytes, str)):
        value = [value]
    if isinstance(value, np.ndarray) and value.dtype.kind == "f":
        arr = np.ascontiguousarray(value, dtype="<f4").ravel()
        return _ld(2, _ld(1, arr.tobytes()))
    if isinstance(value, np.ndarray) and value.dtype.kind in "iu":
        return _ld(3, _ld(1, b"".join(_varint(int(v)) for v in value.ravel())))
    if isinstance(value, float):
        return _ld(2, _ld(1, struct.pack("<f", value)))
    if isinstance(value, (int, np.integer)) and not isinstance(value, bool):
        return _ld(3, _ld(1, _varint(int(value))))
    if isinstance(value, (list, tuple)):
        if all(isinstance(v, (bytes, str)) for v in value):
            return _ld(1, b"".join(_ld(1, v.encode("utf8") if isinstance(v, str) else v) for v in value))
        if all(isinstance(v, float) for v in value):
            return _feature(np.asarray(value, np.float32))
        if all(isinstance(v, (int, np.integer)) for v in value):
            return _feature(np.asarray(value, np.int64))
    raise TypeError(f"unsupported feature value {type(value)}")


def encode_example(features: dict) -> bytes:
    """tf.train.Example(features=tf.train.Features(feature=...)).SerializeToString()
    equivalent (map entries in sorted key order, as protobuf's deterministic mode)."""
    entries = b"".join(_ld(1, _ld(1, k.encode("utf8")) + _ld(2, _feature(v))) for k, v in sorted(features.items()))
    return _ld(1, entries)


def _parse_feature(buf: memoryview):
    pos = 0
    key, pos = _read_varint(buf, pos)
    field = key >> 3
    ln, pos = _read_varint(buf, pos)
    lst = buf[pos:pos + ln]
    if field == 1:  # BytesList
        vals, p = [], 0
        while p < len(lst):
            k, p = _read_varint(lst, p)
            n, p = _read_varint(lst, p)
            vals.append(bytes(lst[p:p + n]))
            p += n
        return vals
    if field == 2:  # FloatList (packed or not)
        out, p = [], 0
        while p < len(lst):
            k, p = _read_varint(lst, p)
            if k & 7 == 2:
                n, p = _read_varint(lst, p)
                out.append(np.frombuffer(lst[p:p + n], dtype="<f4"))
                p += n
            else:
                out.append(np.frombuffer(lst[p:p + 4], dtype="<f4"))
                p += 4
        return np.concatenate(out) if out else np.zeros(0, np.float32)
    if field == 3:  # Int64List
        vals, p = [], 0
        while p < len(lst):
            k, p = _read_varint(lst, p)
            if k & 7 == 2:
                n, p = _read_varint(lst, p)
                end = p + n
                while p < end:
                    v, p = _read_varint(lst, p)
                    vals.append(v - (1 << 64) if v >= 1 << 63 else v)
            else:
                v, p = _read_varint(lst, p)
                vals.append(v - (1 << 64) if v >= 1 << 63 else v)
        return np.asarray(vals, np.int64)
    return None


def decode_example(data: bytes) -> dict:
    """Parse a serialized tf.train.Example into {key: list[bytes] | float32 ndarray | int64 ndarray}."""
    buf = memoryview(data)
    out = {}
    pos = 0
    while pos < len(buf):
        k, pos = _read_varint(buf, pos)
        n, pos = _read_varint(buf, pos)
        feats = buf[pos:pos + n]
        pos += n
        if k >> 3 != 1:
            continue
        fp = 0
        while fp < len(feats):
            k2, fp = _read_varint(feats, fp)
            n2, fp = _read_varint(feats, fp)
            entry = feats[fp:fp + n2]
            fp += n2
            ep, name, val = 0, None, None
            while ep < len(entry):
                k3, ep = _read_varint(entry, ep)
                n3, ep = _read_varint(entry, ep)
                if k3 >> 3 == 1:
                    name = bytes(entry[ep:ep + n3]).decode("utf8")
                elif k3 >> 3 == 2:
                    val = _parse_feature(entry[ep:ep + n3])
                ep += n3
            if name is not None:
                out[name] = val
    return out


# ------------------------------------------------------------------ record framing
def frame(data: bytes) -> bytes:
    ln = struct.pack("<Q", len(data))
    return ln + struct.pack("<I", masked_crc(ln)) + data + struct.pack("<I", masked_crc(data))


class TFRecordWriter:
    """tf.io.TFRecordWriter(path, options="GZIP") equivalent (audiowriter.py:259-277)."""

    def __init__(self, path, compression: str | None = "GZIP"):
        # zlib level 6 = Z_DEFAULT_COMPRESSION, what TF's GZIP writer uses
        self._f = gzip.open(path, "wb", compresslevel=6) if compression == "GZIP" else open(path, "wb")

    def write(self, record: bytes):
        self._f.write(frame(record))

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class ShardReader:
    """One TFRecord shard through the native reader (acfe_tfr_* in libacfe:
    whole-file inflate with libdeflate, hardware CRC-32C); records are
    zero-copy (pointer, length) views valid until close().  ctypes releases
    the GIL inside every call, so reader threads inflate and parse in
    parallel."""

    def __init__(self, path, compression: str | None = "GZIP"):
        from acfe._lib import lib

        self._lib = lib
        self._h = ctypes.c_void_p()
        rc = lib.acfe_tfr_open(str(path).encode(), 1 if compression == "GZIP" else 0, ctypes.byref(self._h))
        if rc < 0:
            self._h = None
            raise IOError(f"cannot open TFRecord shard {path} (rc={rc})")
        self._ptr = ctypes.c_void_p()
        self._len = ctypes.c_uint64()

    def next(self, check_crc=True):
        """(address, length) of the next record, None at a clean end; IOError on
        a truncated / CRC-failing record (nothing after it is readable)."""
        rc = self._lib.acfe_tfr_next(self._h, int(check_crc), ctypes.byref(self._ptr), ctypes.byref(self._len))
        if rc == 1:
            return self._ptr.value, self._len.value
        if rc == 0:
            return None
        raise IOError("corrupt or truncated TFRecord")

    def close(self):
        if self._h is not None:
            self._lib.acfe_tfr_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        self.close()


def read_records(path, compression: str | None = "GZIP", check_crc=True, ignore_errors=False) -> Iterator[bytes]:
    """tf.data.TFRecordDataset(path, compression_type="GZIP") record stream.
    ignore_errors mirrors tf.data.experimental.ignore_errors() (tfdataset.py:226):
    an unreadable file or a corrupt record ends the file instead of raising."""
    try:
        r = ShardReader(path, compression)
    except IOError:
        if ignore_errors:
            return
        raise
    with r:
        while True:
            try:
                rec = r.next(check_crc)
            except IOError:
                if ignore_errors:
                    return
                raise
            if rec is None:
                return
            yield ctypes.string_at(rec[0], rec[1])


def write_records(path, records: Iterable[bytes], compression="GZIP") -> int:
    n = 0
    with TFRecordWriter(path, compression) as w:
        for r in records:
            w.write(r)
            n += 1
    return n


# ------------------------------------------------------------------ the audio schema
def audio_example(raw: np.ndarray, rec_id, track_id, text_tags: str, ebird_tags: str, start_s=0.0, low_sample=0,
                  lat=0.0, lng=0.0, signal_percent=0.0, sample_rate=48000, length=3.0, spectrogram=None) -> bytes:
    """create_tf_example (audiowriter.py:67-174) for one 3 s sample."""
    raw = np.asarray(raw, np.float32).ravel()
    f = {
        "audio/lat": float(lat), "audio/lng": float(lng),
        "audio/rec_id": str(rec_id).encode(), "audio/track_id": str(track_id).encode(),
        "audio/sample_rate": int(sample_rate), "audio/min_freq": -1.0, "audio/max_freq": -1.0,
        "audio/length": float(length), "audio/signal_percent": float(signal_percent),
        "audio/low_sample": int(low_sample), "audio/raw_length": float(len(raw) / sample_rate),
        "audio/start_s": float(start_s), "audio/class/text": text_tags.encode(),
        "audio/class/ebird": ebird_tags.encode(), "audio/raw": raw,
    }
    if spectrogram is not None:
        f["audio/spectogram"] = np.asarray(spectrogram, np.float32).ravel()
    return encode_example(f)


def parse_audio_example(data: bytes, load_raw=True, n_samples=48000 * 3):
    """The fields read_tfrecord takes (tfdataset.py:1005-1060): returns a dict with
    'raw' (float32 [144000]) or 'spectrogram' ([2049, 513]), 'text', 'ebird',
    'rec_id', 'track_id', 'low_sample', 'start_s', 'lat', 'lng', 'signal_percent'."""
    ex = decode_example(data)

    def s(k):
        v = ex.get(k)
        return v[0].decode() if v else ""

    def f(k):
        v = ex.get(k)
        return float(v[0]) if v is not None and len(v) else 0.0

    out = {"text": s("audio/class/text"), "ebird": s("audio/class/ebird"), "rec_id": s("audio/rec_id"),
           "track_id": s("audio/track_id"), "start_s": f("audio/start_s"), "lat": f("audio/lat"),
           "lng": f("audio/lng"), "signal_percent": f("audio/signal_percent"),
           "low_sample": int(ex["audio/low_sample"][0]) if "audio/low_sample" in ex else 0}
    if load_raw:
        raw = ex.get("audio/raw")
        if raw is None or raw.size != n_samples:
            raise ValueError(f"audio/raw must hold {n_samples} floats")
        out["raw"] = raw
    else:
        out["spectrogram"] = ex["audio/spectogram"].reshape(2049, 513)
    return out
