"""16-bit PCM WAV I/O matching `soundfile.write(path, x, 16000)`.

The reference writes every output with `sf.write(path, x, sample_rate)`
(scripts/test.py:165-169). For a `.wav` path and float data, soundfile picks
the default subtype PCM_16, and libsndfile converts each sample as
`(short) lrintf(x * 0x7FFF)`:
- the scale is 0x7FFF, not 0x8000;
- lrintf rounds half to even;
- clipping is off by default (SFC_SET_CLIPPING), so values beyond
  [-1, 32768/32767) wrap modulo 2^16.

The file is the canonical 44-byte header: RIFF/WAVE, a 16-byte `fmt `
chunk (PCM, mono), then `data`.

soundfile / libsndfile are absent here, so the wrap-versus-clip behaviour
for |x| > 1 is unpinned. `clip=True` selects the
saturating variant.
"""
from __future__ import annotations

import os
import struct

import numpy as np


def pcm16(x: np.ndarray, clip: bool = False) -> np.ndarray:
    """float -> int16 exactly as libsndfile's f2s conversion (lrintf(x * 0x7FFF))."""
    y = np.rint(np.asarray(x, np.float32) * np.float32(0x7FFF))     # float32 product, ties to even
    if clip:
        y = np.clip(y, -32768, 32767)
    return y.astype(np.int64).astype(np.int16)                      # wrap modulo 2^16


def write_wav(path: str, x: np.ndarray, sample_rate: int = 16000, clip: bool = False) -> None:
    s = pcm16(np.asarray(x).reshape(-1), clip=clip)
    data = s.astype('<i2').tobytes()
    hdr = b'RIFF' + struct.pack('<I', 36 + len(data)) + b'WAVE'
    hdr += b'fmt ' + struct.pack('<IHHIIHH', 16, 1, 1, sample_rate, sample_rate * 2, 2, 16)
    hdr += b'data' + struct.pack('<I', len(data))
    tmp = path + '.tmp'
    with open(tmp, 'wb') as fh:
        fh.write(hdr + data)
    os.replace(tmp, path)


def read_wav(path: str):
    """(samples as float32 in [-1, 1), sample_rate) for PCM16 / float32 mono
    or multichannel WAV; sf.read's default float64 scaling is 1/32768."""
    raw = open(path, 'rb').read()
    if raw[:4] != b'RIFF' or raw[8:12] != b'WAVE':
        raise ValueError(f'{path}: not a RIFF/WAVE file')
    p, fmt, data = 12, None, None
    while p + 8 <= len(raw):
        cid, size = raw[p:p + 4], struct.unpack('<I', raw[p + 4:p + 8])[0]
        body = raw[p + 8:p + 8 + size]
        if cid == b'fmt ':
            fmt = struct.unpack('<HHIIHH', body[:16])
        elif cid == b'data':
            data = body
        p += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise ValueError(f'{path}: missing fmt / data chunk')
    tag, ch, sr, _, _, bits = fmt
    if tag == 1 and bits == 16:
        a = np.frombuffer(data, '<i2').astype(np.float32) / 32768.0
    elif tag == 3 and bits == 32:
        a = np.frombuffer(data, '<f4').astype(np.float32)
    else:
        raise ValueError(f'{path}: unsupported WAV format tag {tag} / {bits} bits')
    return (a.reshape(-1, ch) if ch > 1 else a), sr
