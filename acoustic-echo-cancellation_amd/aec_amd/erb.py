"""ERB filterbank — host-side drop-in for the reference's
``EquivalentRectangularBandwidth`` (Stage2_lhm/scripts/network/ERB.py:10-71).

Init-time only (float64 NumPy).  ``filters`` is the [nfreqs, bands] cosine
filterbank; like the reference, the 34-band version with low/high-pass edge
filters is built and discarded (ERB.py:60-71 return only ``cos_filts``).
The device path consumes the float32 cast of ``filters`` in two sparse views
(see csrc/aec_tables.h).
"""
from __future__ import annotations

import numpy as np


class EquivalentRectangularBandwidth:
    EarQ = 9.265      # Glasberg & Moore ERB Q          (ERB.py:17)
    minBW = 24.7      # minimum bandwidth in Hz          (ERB.py:18)

    def __init__(self, nfreqs, sample_rate, total_erb_bands, low_freq, max_freq):
        if low_freq is None:
            low_freq = 20
        if max_freq is None:
            max_freq = sample_rate // 2
        self.nfreqs = nfreqs
        self.freqs = np.linspace(0, max_freq, nfreqs)                       # bin centre (Hz)
        lims = np.linspace(self.freq2erb(low_freq), self.freq2erb(max_freq), total_erb_bands + 2)
        self.cutoffs = self.erb2freq(lims)                                   # band edges (Hz)
        self.filters = self._cos_lobes(total_erb_bands)

    def freq2erb(self, f):
        return self.EarQ * np.log(1 + f / (self.minBW * self.EarQ))

    def erb2freq(self, e):
        return (np.exp(e / self.EarQ) - 1) * self.minBW * self.EarQ

    def _cos_lobes(self, bands):
        """Band i is a half-cosine lobe spanning cutoffs i .. i+2 (50 % overlap),
        evaluated on the bins strictly inside that interval (ERB.py:46-58)."""
        f = self.freqs
        out = np.zeros([self.nfreqs, bands])
        for i in range(bands):
            lo, hi = self.cutoffs[i], self.cutoffs[i + 2]
            first = np.min(np.where(f > lo))
            last = np.max(np.where(f < hi))
            e_lo, e_hi = self.freq2erb(lo), self.freq2erb(hi)
            centre = (e_lo + e_hi) / 2
            width = e_hi - e_lo
            out[first:last + 1, i] = np.cos((self.freq2erb(f[first:last + 1]) - centre) / width * np.pi)
        return out


def erb_matrix(nfreqs=257, sample_rate=16000, bands=32, low_freq=0, max_freq=8000):
    """float64 [nfreqs, bands] filterbank for erb_conf (scripts/configs.py:21-27)."""
    return EquivalentRectangularBandwidth(nfreqs, sample_rate, bands, low_freq, max_freq).filters
