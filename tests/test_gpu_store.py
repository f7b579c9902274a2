"""Index files (ngsSaveIndex / ngsLoadIndex): a loaded index is the saved
one, array for array (ngsIndexDigest: the gram CSR and the wildcard answer are rebuilt from the
interned library), answers every query exactly like it, keeps its validChar set, and bad files
are refused."""
import ctypes as C
import os
import random

import pytest

import stringsearchlib_amd as ssl
from stringsearchlib_amd import _native

pytestmark = pytest.mark.gpu


def _digest(idx):
    out = (C.c_uint64 * 17)()
    assert _native.lib().ngsIndexDigest(idx.handle, out, 17) == 17
    return list(out)


def _messy(rng, n, rs):
    alpha = "ABCDEFabcdef0123 .-_#"
    words = []
    for _ in range(n * rs):
        r = rng.random()
        words.append(None if r < 0.04 else "".join(rng.choice(alpha) for _ in range(rng.randint(1, 16))))
    return words, [rng.choice([1.0, 0.5, 2.0, 0.0, -0.5, 0.75]) for _ in words]


@pytest.mark.parametrize("kind", ["narrow", "aliases", "gram2", "wide"])
def test_save_load_roundtrip(tmp_path, kind):
    rng = random.Random(len(kind))
    if kind == "narrow":
        words, wts, _ = ssl.synth.gen_corpus(30000, seed=3)
        gi = ssl.StringIndex(words, 1, wts)
    elif kind == "aliases":
        words, wts = _messy(rng, 5000, 3)
        words = [None if w is None else w.encode("latin-1") for w in words]
        gi = ssl.StringIndex(words, 3, wts)
    elif kind == "gram2":
        words, wts = _messy(rng, 5000, 1)
        words = [None if w is None else w.encode("latin-1") for w in words]
        gi = ssl.StringIndex(words, 1, wts, gram_size=2)
    else:
        words, wts = _messy(rng, 4000, 2)
        gi = ssl.WideStringIndex(words, 2, wts, gram_size=2)
    if kind == "narrow":
        gi.set_valid_char(b".%$ @0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ")  # travels with the file
    path = str(tmp_path / f"{kind}.ngs")
    gi.save(path)
    cls = type(gi)
    li = cls.load(path)
    assert _digest(li) == _digest(gi)
    assert li.size() == gi.size() and li.lib_size() == gi.lib_size() and li.num_keys() == gi.num_keys()
    keys = [w for w in words if w]
    qs = [rng.choice(keys) for _ in range(120)] + [k[:5] for k in keys[:40:4]]
    qs += ["*", ""] if kind == "wide" else [b"*", b""]
    for thr, limit in [(0.3, 100), (0.0, 10), (0.7, 3)]:
        assert li.score_batch(qs, thr, limit) == gi.score_batch(qs, thr, limit), (kind, thr, limit)
    li.dispose()
    gi.dispose()


def test_load_refuses_bad_files(tmp_path):
    L = _native.lib()
    missing = str(tmp_path / "missing.ngs")
    assert L.ngsLoadIndex(os.fsencode(missing)) == 0
    junk = tmp_path / "junk.ngs"
    junk.write_bytes(b"NGSIDX01" + b"\x01" * 64)
    assert L.ngsLoadIndex(os.fsencode(str(junk))) == 0
    words, wts, _ = ssl.synth.gen_corpus(2000, seed=9)
    gi = ssl.StringIndex(words, 1, wts)
    good = tmp_path / "good.ngs"
    gi.save(str(good))
    data = good.read_bytes()
    (tmp_path / "cut.ngs").write_bytes(data[: len(data) // 2])  # truncated
    assert L.ngsLoadIndex(os.fsencode(str(tmp_path / "cut.ngs"))) == 0
    assert L.ngsSaveIndex(987654, os.fsencode(str(tmp_path / "x.ngs"))) == -1
    with pytest.raises(TypeError):
        ssl.WideStringIndex.load(str(good))
    # files whose counts agree but whose contents are inconsistent: each refused
    for name, bad in _corruptions(data).items():
        f = tmp_path / f"{name}.ngs"
        f.write_bytes(bad)
        assert L.ngsLoadIndex(os.fsencode(str(f))) == 0, name
    gi.dispose()


def _corruptions(data: bytes) -> dict:
    """Variants of a saved index file (layout: ngs_abi.cpp, "NGSIDX01" | 9 u32 scalars | 8 u32
    validChar words | arrays as u64 count + elements) that keep every count consistent."""
    import struct
    pos = 8 + 9 * 4 + 8 * 4
    arrays = {}
    for name, width in [("term_off", 8), ("term_bytes", 1), ("tk_off", 4), ("tk", 8), ("key_off", 8),
                        ("key_bytes", 1), ("wild_w", 4)]:
        (n,) = struct.unpack_from("<Q", data, pos)
        arrays[name] = (pos + 8, n, width)
        pos += 8 + n * width
    assert pos == len(data)
    out = {}

    def patch(off, fmt, val):
        b = bytearray(data)
        struct.pack_into(fmt, b, off, val)
        return bytes(b)

    o, n, _ = arrays["term_off"]
    out["term_off_descending"] = patch(o + 8 * (n // 2), "<Q", 0)
    o, n, _ = arrays["key_off"]
    out["key_off_descending"] = patch(o + 8 * (n // 3), "<Q", 0)
    o, n, _ = arrays["tk_off"]
    out["tk_off_first_nonzero"] = patch(o, "<I", 1)
    o, n, _ = arrays["key_bytes"]
    out["key_without_nul"] = patch(o + n - 1, "<B", ord("X"))
    out["short_term_len"] = patch(8 + 3 * 4, "<I", 5)
    out["gram_mode"] = patch(8 + 2 * 4, "<I", 1)
    (n_short,) = struct.unpack_from("<I", data, 8 + 7 * 4)
    out["n_short"] = patch(8 + 7 * 4, "<I", n_short + 1)
    return out
