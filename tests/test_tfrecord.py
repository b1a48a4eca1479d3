"""TFRecord / tf.train.Example codec (no TensorFlow): CRC-32C vectors, framing,
GZIP round trip, corruption handling, and a cross-check of the hand-written
wire format against the protobuf runtime using the published
tensorflow/core/example/{example,feature}.proto message layout."""
import gzip
import struct

import numpy as np
import pytest

import tfrecord as tfr


def test_crc32c_vectors():
    # RFC 3720 B.4 / common check values
    assert tfr._crc32c(b"123456789") == 0xE3069283
    assert tfr._crc32c(bytes(32)) == 0x8A9136AA
    assert tfr._crc32c(b"\xff" * 32) == 0x62A8AB43
    assert tfr._crc32c(bytes(range(32))) == 0x46DD794E


def _example_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="tfr_example_test.proto", package="tensorflow", syntax="proto3")

    def msg(name, fields, nested=None, oneof=None):
        m = fdp.message_type.add(name=name)
        if oneof:
            m.oneof_decl.add(name=oneof)
        for fname, num, typ, label, tname, in_oneof in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
            if in_oneof:
                f.oneof_index = 0
        if nested:
            nested(m)
        return m

    R, O = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, F.TYPE_BYTES, R, None, False)])
    msg("FloatList", [("value", 1, F.TYPE_FLOAT, R, None, False)])
    msg("Int64List", [("value", 1, F.TYPE_INT64, R, None, False)])
    msg("Feature", [("bytes_list", 1, F.TYPE_MESSAGE, O, ".tensorflow.BytesList", True),
                    ("float_list", 2, F.TYPE_MESSAGE, O, ".tensorflow.FloatList", True),
                    ("int64_list", 3, F.TYPE_MESSAGE, O, ".tensorflow.Int64List", True)], oneof="kind")

    def entry(m):
        e = m.nested_type.add(name="FeatureEntry")
        e.field.add(name="key", number=1, type=F.TYPE_STRING, label=O)
        e.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=O, type_name=".tensorflow.Feature")
        e.options.map_entry = True

    msg("Features", [("feature", 1, F.TYPE_MESSAGE, R, ".tensorflow.Features.FeatureEntry", False)], nested=entry)
    msg("Example", [("features", 1, F.TYPE_MESSAGE, O, ".tensorflow.Features", False)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tensorflow.Example"))


def _sample(rng):
    raw = rng.standard_normal(144000).astype(np.float32)
    return raw, tfr.audio_example(raw, 1234, "7 8", "bird", "morepo2", start_s=1.5, low_sample=1, lat=-43.5,
                                  lng=172.6, signal_percent=0.25)


def test_example_roundtrip_and_protobuf_crosscheck():
    Example = _example_class()
    raw, data = _sample(np.random.default_rng(0))
    # our encoder -> protobuf parser
    ex = Example()
    ex.ParseFromString(data)
    feat = ex.features.feature
    assert np.array_equal(np.asarray(feat["audio/raw"].float_list.value, np.float32), raw)
    assert feat["audio/class/text"].bytes_list.value[0] == b"bird"
    assert feat["audio/low_sample"].int64_list.value[0] == 1
    assert abs(feat["audio/start_s"].float_list.value[0] - 1.5) < 1e-7
    # protobuf serializer -> our decoder (including negative int64 and multi-bytes)
    ex2 = Example()
    ex2.features.feature["a"].int64_list.value.extend([-5, 3, 1 << 40])
    ex2.features.feature["b"].bytes_list.value.extend([b"x", b"yz"])
    ex2.features.feature["c"].float_list.value.extend([0.5, -2.25])
    d = tfr.decode_example(ex2.SerializeToString())
    assert d["a"].tolist() == [-5, 3, 1 << 40] and d["b"] == [b"x", b"yz"] and d["c"].tolist() == [0.5, -2.25]
    p = tfr.parse_audio_example(data)
    assert np.array_equal(p["raw"], raw) and p["ebird"] == "morepo2" and p["rec_id"] == "1234"
    assert p["low_sample"] == 1 and p["track_id"] == "7 8"


def test_gzip_file_roundtrip_and_corruption(tmp_path):
    rng = np.random.default_rng(1)
    recs = [_sample(rng)[1] for _ in range(5)]
    path = tmp_path / "a.tfrecord"
    assert tfr.write_records(path, recs) == 5
    assert list(tfr.read_records(path)) == recs
    raw = bytearray(gzip.decompress(path.read_bytes()))
    # the first record's header CRC is the masked CRC of its length field
    assert struct.unpack("<I", raw[8:12])[0] == tfr.masked_crc(bytes(raw[:8]))
    raw[200] ^= 0xFF  # flip a data byte of record 0
    bad = tmp_path / "bad.tfrecord"
    bad.write_bytes(gzip.compress(bytes(raw)))
    with pytest.raises(IOError):
        list(tfr.read_records(bad))
    assert list(tfr.read_records(bad, ignore_errors=True)) == []
    # truncated file: ignore_errors keeps the intact prefix
    trunc = tmp_path / "trunc.tfrecord"
    full = gzip.decompress(path.read_bytes())
    trunc.write_bytes(gzip.compress(full[: len(full) - 10]))
    assert len(list(tfr.read_records(trunc, ignore_errors=True))) == 4


def test_empty_file(tmp_path):
    p = tmp_path / "e.tfrecord"
    tfr.write_records(p, [])
    assert list(tfr.read_records(p)) == []
