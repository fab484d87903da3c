"""The reference's shipped Torch7 vocabulary caches (BiCNN/binary_map*) through the
plain-data Torch7 reader (mpit_amd/utils/t7.py), and BiCNN's -preloadBinary on them."""
import os
import struct

import pytest

from mpit_amd.utils import t7

REF = "/root/reference/BiCNN"
needs_ref = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "binary_mapWordStr2WordIdx")),
                               reason="reference checkout with the BiCNN vocabulary caches not present")


@needs_ref
def test_shipped_vocabulary_maps_are_inverse():
    s2i = t7.load(os.path.join(REF, "binary_mapWordStr2WordIdx"))
    i2s = t7.load(os.path.join(REF, "binary_mapWordIdx2WordStr"))
    assert len(s2i) == len(i2s) == 22354
    assert sorted(i2s) == list(range(1, 22355))
    assert all(i2s[i] == w for w, i in s2i.items())
    assert all(s2i[w] == i for i, w in i2s.items())
    assert s2i["SENTBEGIN"] == 1 and s2i["SENTEND"] == 2 and i2s[1] == "SENTBEGIN" and i2s[2] == "SENTEND"


@needs_ref
def test_bicnn_preload_binary_builds_vocabulary_from_t7_maps():
    from mpit_amd.apps import bicnn
    from mpit_amd.apps.qa_data import load_t7_vocab

    a = bicnn.build_args(["-preloadBinary", "-binaryDir", REF, "-synthetic", "20"])
    data = bicnn.load_data(a)
    vocab = load_t7_vocab(REF)
    assert len(data.word2idx) == 22355 and data.word2idx["<pad>"] == 0
    assert all(data.word2idx[w] == i for w, i in vocab.items())
    emb = data.embedding_matrix()
    assert emb.shape == (22355, a.embeddingDim) and float(emb[:3].abs().sum()) == 0.0
    # every token of the prepared data is a vocabulary id
    ids = {i for _, q, ans in data.train for i in q + ans}
    assert ids <= set(range(1, 22355)) and len(data.answers) == 20


def test_t7_roundtrip_and_shared_tables():
    v = {1: "a", "b": 2.5, "c": {"x": True, "y": None}, "n": -3}
    assert t7.loads(t7.dumps(v)) == v
    # a table referenced twice (Torch7 back-reference) is the same object
    inner = struct.pack("<iii", 3, 2, 1) + struct.pack("<id", 1, 7.0) + struct.pack("<ii", 2, 1) + b"z"
    blob = struct.pack("<iii", 3, 1, 2) + struct.pack("<id", 1, 1.0) + inner + struct.pack("<id", 1, 2.0) + struct.pack("<ii", 3, 2)
    out = t7.loads(blob)
    assert out[1] is out[2] and out[1] == {7: "z"}


@pytest.mark.parametrize("tag", [4, 6, 7, 8])
def test_t7_refuses_objects_and_functions(tag):
    blob = struct.pack("<iii", 3, 1, 1) + struct.pack("<id", 1, 1.0) + struct.pack("<i", tag) + b"\0" * 16
    with pytest.raises(t7.T7RefusedObject):
        t7.loads(blob)


def test_t7_rejects_truncated_and_trailing():
    blob = t7.dumps({"k": "v"})
    with pytest.raises(ValueError):
        t7.loads(blob[:-1])
    with pytest.raises(ValueError):
        t7.loads(blob + b"\0")


@needs_ref
def test_bicnn_preload_binary_prefers_the_binary_file(tmp_path, capsys):
    """-preloadBinary takes --binaryFile when it exists, even next to the Torch7 maps; the
    vocabulary-only mode says loudly that its questions / answers are synthetic."""
    from mpit_amd.apps import bicnn
    from mpit_amd.apps.qa_data import save_binary, synthetic_qa

    f = str(tmp_path / "qa.pt")
    save_binary(synthetic_qa(n_answers=7, pool=5, n_train=50, n_valid=10, emb_dim=16, conv_width=2), f)
    a = bicnn.build_args(["-preloadBinary", "-binaryDir", REF, "-binaryFile", f, "-embeddingDim", "16"])
    assert len(bicnn.load_data(a).answers) == 7
    assert "SYNTHETIC" not in capsys.readouterr().err
    a = bicnn.build_args(["-preloadBinary", "-binaryDir", REF, "-binaryFile", str(tmp_path / "none.pt"),
                          "-synthetic", "20"])
    assert len(bicnn.load_data(a).answers) == 20
    assert "SYNTHETIC" in capsys.readouterr().err
