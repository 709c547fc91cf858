"""HDF5 container of the reference's test sets.

libhdf5 / h5py are absent here, so parity against them is unpinned. These
tests pin:
- the on-disk constants and structures the specification fixes;
- writer -> reader round trips over the shapes the reference uses: ragged
  per-utterance lengths, multi-chunk datasets, more than 256 groups (a
  multi-level group B-tree) and empty datasets;
- the chunk size h5py's `chunks=True` picks.
"""
import os
import struct
import zlib

import numpy as np
import pytest

from aec_amd import h5lite


def _utts(lens, seed=0):
    rng = np.random.default_rng(seed)
    return [{k: rng.standard_normal(n).astype(np.float32) for k in h5lite.SIGNALS} for n in lens]


@pytest.mark.parametrize('chunks', [True, False])
def test_roundtrip_ragged(tmp_path, chunks):
    lens = [160000, 64123, 255, 1, 513, 191999]
    utts = _utts(lens)
    p = str(tmp_path / 'test.ex')
    h5lite.write_utterances(p, utts, chunks=chunks)
    with h5lite.File(p) as f:
        assert len(f) == len(lens)
        assert sorted(f.keys(), key=int) == [str(i) for i in range(len(lens))]
        for i, u in enumerate(utts):
            e = h5lite.read_utterance(f, i)
            assert e['n_samples'] == lens[i]
            for k in h5lite.SIGNALS:
                assert e[k].dtype == np.float32 and e[k].shape == (lens[i],)
                assert np.array_equal(e[k], u[k])


def test_many_groups_multilevel_btree(tmp_path):
    lens = [100 + (i * 37) % 300 for i in range(300)]        # > 256 names: B-tree of depth 2
    utts = _utts(lens, seed=1)
    p = str(tmp_path / 'big.ex')
    h5lite.write_utterances(p, utts)
    with h5lite.File(p) as f:
        assert len(f) == 300
        for i in [0, 7, 8, 255, 256, 299]:
            assert np.array_equal(np.array(f[str(i)]['echo']), utts[i]['echo'])
        assert np.array_equal(np.array(f['123/nearend_mic']), utts[123]['nearend_mic'])


def test_superblock_and_structures(tmp_path):
    p = str(tmp_path / 'one.ex')
    h5lite.write_utterances(p, _utts([3000]))
    raw = open(p, 'rb').read()
    assert raw[:8] == b'\x89HDF\r\n\x1a\n'
    assert raw[8] == 0                                        # superblock version 0
    assert raw[13] == 8 and raw[14] == 8                      # offset / length sizes
    leafK, internK, flags = struct.unpack('<HHI', raw[16:24])
    assert (leafK, internK, flags) == (4, 16, 0)
    base, fs, eof, drv = struct.unpack('<QQQQ', raw[24:56])
    assert base == 0 and fs == h5lite.UNDEF and drv == h5lite.UNDEF and eof == len(raw)
    assert b'TREE' in raw and b'SNOD' in raw and b'HEAP' in raw
    assert raw.count(b'nearend_speech\0') == 1


def test_h5py_default_chunk_size():
    # h5py guess_chunk for 1-D float32 data (halving until near the target)
    # 160000 x 4 B = 625 KiB -> target 16 KiB * 2**log10(0.61) = 13.8 KiB; 5000 x 4 B is within 50 %
    assert h5lite.default_chunk(160000) == 5000
    assert h5lite.default_chunk(100) == 100
    assert h5lite.default_chunk(0) == 1024
    for n in [1, 255, 16000, 160000, 1_000_000]:
        c = h5lite.default_chunk(n)
        assert 1 <= c <= max(n, 1) and c * 4 < 1024 * 1024


def test_filters_deflate_shuffle():
    a = np.arange(1000, dtype=np.float32)
    shuf = a.view(np.uint8).reshape(-1, 4).T.reshape(-1).tobytes()
    comp = zlib.compress(shuf)
    out = h5lite._unfilter(comp, [(2, []), (1, [6])], 0, 4)
    assert np.array_equal(np.frombuffer(out, np.float32), a)
    # mask bit set: that filter was skipped at write time
    out2 = h5lite._unfilter(zlib.compress(a.tobytes()), [(2, []), (1, [6])], 0b01, 4)
    assert np.array_equal(np.frombuffer(out2, np.float32), a)


def test_rejects_non_hdf5_and_latest(tmp_path):
    p = tmp_path / 'x.ex'
    p.write_bytes(b'not an hdf5 file' * 10)
    with pytest.raises(h5lite.H5Error):
        h5lite.File(str(p))
    q = tmp_path / 'v2.ex'
    q.write_bytes(h5lite.SIGNATURE + bytes([2]) + b'\0' * 100)
    with pytest.raises(h5lite.H5Error, match='superblock version 2'):
        h5lite.File(str(q))


# ---------------------------------------------------------- libhdf5-written files
FOREIGN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'foreign')


def test_reads_libhdf5_file_with_user_block():
    """A MATLAB 7.3 file written by libhdf5 (superblock at 512 behind a user
    block; addresses relative to it): the variable equals what scipy's MATLAB
    v5 reader returns for the same variable saved by the same MATLAB."""
    import scipy.io as sio
    with open(os.path.join(FOREIGN, 'testhdf5_7.4_GLNX86.mat'), 'rb') as fh:
        raw = fh.read()
    assert raw[512:520] == h5lite.SIGNATURE and raw[:8] != h5lite.SIGNATURE
    f = h5lite.File(os.path.join(FOREIGN, 'testhdf5_7.4_GLNX86.mat'))
    try:
        assert f.keys() == ['testdouble']
        got = f['testdouble'].read()
    finally:
        f.close()
    exp = sio.loadmat(os.path.join(FOREIGN, 'testdouble_7.4_GLNX86.mat'))['testdouble']
    assert got.dtype == np.float64 and got.shape == exp.T.shape     # HDF5 MATLAB arrays are stored transposed
    assert np.array_equal(got, exp.T)
    assert np.array_equal(got[:, 0], np.linspace(0, 2 * np.pi, 9))


def test_reads_hdf5_example_files():
    """libhdf5-written example files (PyTables' test data): contiguous
    float16/32/64, big-endian int32 (h5_write: data[i][j] = i + j) and a
    chunked, extended dataset (h5_extend)."""
    with h5lite.File(os.path.join(FOREIGN, 'float.h5')) as f:
        ij = np.add.outer(np.arange(5), np.arange(6))
        for k, dt in (('float16', np.float16), ('float32', np.float32), ('float64', np.float64)):
            a = f[k].read()
            assert a.dtype == dt and np.array_equal(a, ij.astype(dt))
    with h5lite.File(os.path.join(FOREIGN, 'smpl_i32be.h5')) as f:
        a = f['TestArray'].read()
        assert a.dtype == np.int32 and np.array_equal(a, np.add.outer(np.arange(6), np.arange(5)))
    with h5lite.File(os.path.join(FOREIGN, 'smpl_SDSextendible.h5')) as f:
        ds = f['ExtendibleArray']
        assert ds._layout[0] == 'chunked'
        a = ds.read()
    exp = np.zeros((10, 5), np.int32)
    exp[:3, :3] = 1
    exp[:2, 3:] = 3
    exp[3:, 0] = 2
    assert np.array_equal(a, exp)
