"""ctypes binding of libaec_hip.so (C ABI declared in include/aec_hip.h).

The HIP library is the ONLY compute path: there is no CPU fallback.  If the
library has not been built (``python -c "import __graft_entry__ as g; g.build()"``)
every entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# AEC_HIP_LIB: alternative build of the same library (A/B timing experiments)
_DEFAULT_LIB = os.path.join(_HERE, 'libaec_hip.so')
LIB_PATH = os.environ.get('AEC_HIP_LIB') or _DEFAULT_LIB

# aec_status codes (include/aec_hip.h)
AEC_OK = 0
AEC_ERR_INVALID_ARG = 1
AEC_ERR_OOM = 2
AEC_ERR_HIP = 3
AEC_ERR_UNSUPPORTED = 4
_STATUS = {0: 'AEC_OK', 1: 'AEC_ERR_INVALID_ARG', 2: 'AEC_ERR_OOM', 3: 'AEC_ERR_HIP', 4: 'AEC_ERR_UNSUPPORTED'}

# every symbol include/aec_hip.h declares
EXPORTS = ('aec_weights_count', 'aec_create', 'aec_set_weights', 'aec_set_erb', 'aec_process', 'aec_process_siglens',
           'aec_prepare', 'aec_prepare_siglens', 'aec_process_prepared',
           'aec_stream_open', 'aec_stream_reset', 'aec_stream_step',
           'aec_set_debug', 'aec_debug_copy', 'aec_profile_enable', 'aec_profile_read',
           'aec_erb_tables_check', 'aec_num_frames', 'aec_out_len', 'aec_last_error', 'aec_destroy',
           'aec_set_weights_device', 'aec_train_forward', 'aec_train_backward', 'aec_train_generation',
           'aec_adam_step', 'aec_adam_step_multi', 'aec_build_info')


# every symbol include/aec_crn.h declares
CRN_EXPORTS = ('aec_crn_param_count', 'aec_crn_create', 'aec_crn_set_params', 'aec_crn_process', 'aec_crn_stft',
               'aec_crn_error_spec',
               'aec_crn_stream_open', 'aec_crn_stream_reset', 'aec_crn_stream_step',
               'aec_crn_stream_set_graph', 'aec_crn_stream_stats', 'aec_crn_profile_enable', 'aec_crn_profile_read', 'aec_crn_last_error', 'aec_crn_destroy')


class CrnConfig(ctypes.Structure):
    """aec_crn_config (include/aec_crn.h)."""
    _fields_ = [('version', ctypes.c_int32), ('n_layers', ctypes.c_int32),
                ('conv_channels', ctypes.c_int32 * 9), ('hidden_dim', ctypes.c_int32),
                ('rnn_layers', ctypes.c_int32), ('use_cbn', ctypes.c_int32),
                ('masking_mode', ctypes.c_int32), ('dtype', ctypes.c_int32),
                ('nlms_taps', ctypes.c_int32), ('nlms_mu', ctypes.c_float), ('nlms_beta', ctypes.c_float),
                ('nlms_delta', ctypes.c_float)]


class AecConfig(ctypes.Structure):
    _fields_ = [('win_size', ctypes.c_int32), ('hop_size', ctypes.c_int32),
                ('erb_bands', ctypes.c_int32), ('nlms_taps', ctypes.c_int32),
                ('nlms_mu', ctypes.c_float), ('nlms_beta', ctypes.c_float),
                ('nlms_delta', ctypes.c_float), ('reserved', ctypes.c_int32)]


_lib = None


def load():
    """Load (once) and return the ctypes library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'libaec_hip.so not found at {LIB_PATH}: build it first '
                           '(python -c "import __graft_entry__ as g; g.build()"); '
                           'there is no CPU fallback')
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    lib.aec_weights_count.argtypes = [ctypes.c_int32]
    lib.aec_weights_count.restype = ctypes.c_size_t
    lib.aec_create.argtypes = [ctypes.POINTER(AecConfig), P, ctypes.c_size_t, P, ctypes.c_int32,
                               ctypes.POINTER(P)]
    lib.aec_create.restype = ctypes.c_int
    lib.aec_set_weights.argtypes = [P, P, ctypes.c_size_t]
    lib.aec_set_weights.restype = ctypes.c_int
    lib.aec_set_erb.argtypes = [P, P]
    lib.aec_set_erb.restype = ctypes.c_int
    lib.aec_process.argtypes = [P, P, P, P, P, ctypes.c_int32, ctypes.c_int64, P, ctypes.c_int64, P, P]
    lib.aec_process.restype = ctypes.c_int
    lib.aec_process_siglens.argtypes = [P, P, P, P, P, ctypes.c_int32, ctypes.c_int64, P, ctypes.c_int64, P, P]
    lib.aec_process_siglens.restype = ctypes.c_int
    lib.aec_prepare.argtypes = [P, P, P, P, P, ctypes.c_int32, ctypes.c_int64, P, ctypes.POINTER(ctypes.c_uint64)]
    lib.aec_prepare.restype = ctypes.c_int
    lib.aec_prepare_siglens.argtypes = [P, P, P, P, P, ctypes.c_int32, ctypes.c_int64, P,
                                        ctypes.POINTER(ctypes.c_uint64)]
    lib.aec_prepare_siglens.restype = ctypes.c_int
    if LIB_PATH != _DEFAULT_LIB and not hasattr(lib, 'aec_process_prepared'):
        pass                                   # an older A/B build (AEC_HIP_LIB) without the symbol
    else:
        lib.aec_process_prepared.argtypes = [P, ctypes.c_uint64, P, P, P, P, ctypes.c_int32, ctypes.c_int64, P,
                                             ctypes.c_int64, P, P]
        lib.aec_process_prepared.restype = ctypes.c_int
    lib.aec_stream_open.argtypes = [P, ctypes.c_int32]
    lib.aec_stream_open.restype = ctypes.c_int
    lib.aec_stream_reset.argtypes = [P, ctypes.c_int32, P]
    lib.aec_stream_reset.restype = ctypes.c_int
    lib.aec_stream_step.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_int64, P]
    lib.aec_stream_step.restype = ctypes.c_int
    lib.aec_set_debug.argtypes = [P, ctypes.c_int32]
    lib.aec_set_debug.restype = ctypes.c_int
    lib.aec_debug_copy.argtypes = [P, ctypes.c_int32, P, ctypes.c_size_t, P]
    lib.aec_debug_copy.restype = ctypes.c_int
    lib.aec_profile_enable.argtypes = [P, ctypes.c_int32]
    lib.aec_profile_enable.restype = ctypes.c_int
    lib.aec_profile_read.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    lib.aec_profile_read.restype = ctypes.c_int
    lib.aec_erb_tables_check.argtypes = [P, P, P, P, P, ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_int32)]
    lib.aec_erb_tables_check.restype = ctypes.c_int
    lib.aec_num_frames.argtypes = [ctypes.c_int64]
    lib.aec_num_frames.restype = ctypes.c_int64
    lib.aec_out_len.argtypes = [ctypes.c_int64]
    lib.aec_out_len.restype = ctypes.c_int64
    if LIB_PATH == _DEFAULT_LIB or hasattr(lib, 'aec_build_info'):
        lib.aec_build_info.argtypes = []
        lib.aec_build_info.restype = ctypes.c_char_p
    lib.aec_last_error.argtypes = [P]
    lib.aec_last_error.restype = ctypes.c_char_p
    lib.aec_destroy.argtypes = [P]
    lib.aec_destroy.restype = None
    lib.aec_set_weights_device.argtypes = [P, P, ctypes.c_size_t, P]
    lib.aec_set_weights_device.restype = ctypes.c_int
    lib.aec_train_forward.argtypes = [P, P, P, P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, P, ctypes.c_int64,
                                      P, P]
    lib.aec_train_forward.restype = ctypes.c_int
    lib.aec_train_backward.argtypes = [P, P, P, P]
    lib.aec_train_backward.restype = ctypes.c_int
    lib.aec_train_generation.argtypes = [P]
    lib.aec_train_generation.restype = ctypes.c_int64
    F = ctypes.c_float
    lib.aec_adam_step.argtypes = [P, P, P, P, P, ctypes.c_size_t, ctypes.c_int64, F, F, F, F, F, P]
    lib.aec_adam_step.restype = ctypes.c_int
    lib.aec_adam_step_multi.argtypes = [P, P, P, P, P, P, P, ctypes.c_int32, F, F, F, F, F, P]
    lib.aec_adam_step_multi.restype = ctypes.c_int
    # DCCRN (include/aec_crn.h)
    lib.aec_crn_param_count.argtypes = [ctypes.POINTER(CrnConfig)]
    lib.aec_crn_param_count.restype = ctypes.c_size_t
    lib.aec_crn_create.argtypes = [ctypes.POINTER(CrnConfig), P, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(P)]
    lib.aec_crn_create.restype = ctypes.c_int
    lib.aec_crn_set_params.argtypes = [P, P, ctypes.c_size_t]
    lib.aec_crn_set_params.restype = ctypes.c_int
    lib.aec_crn_process.argtypes = [P, P, P, P, ctypes.c_int32, ctypes.c_int64, P, ctypes.c_int64, P, P, P]
    lib.aec_crn_process.restype = ctypes.c_int
    lib.aec_crn_stft.argtypes = [P, P, P, ctypes.c_int32, ctypes.c_int64, P, P]
    lib.aec_crn_stft.restype = ctypes.c_int
    lib.aec_crn_error_spec.argtypes = [P, P, P]
    lib.aec_crn_error_spec.restype = ctypes.c_int
    lib.aec_crn_stream_open.argtypes = [P, ctypes.c_int32]
    lib.aec_crn_stream_open.restype = ctypes.c_int
    lib.aec_crn_stream_reset.argtypes = [P, ctypes.c_int32, P]
    lib.aec_crn_stream_reset.restype = ctypes.c_int
    lib.aec_crn_stream_step.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_int64, P]
    lib.aec_crn_stream_step.restype = ctypes.c_int
    lib.aec_crn_stream_set_graph.argtypes = [P, ctypes.c_int32]
    lib.aec_crn_stream_set_graph.restype = ctypes.c_int
    lib.aec_crn_stream_stats.argtypes = [P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int64)]
    lib.aec_crn_stream_stats.restype = ctypes.c_int
    lib.aec_crn_profile_enable.argtypes = [P, ctypes.c_int32]
    lib.aec_crn_profile_enable.restype = ctypes.c_int
    lib.aec_crn_profile_read.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    lib.aec_crn_profile_read.restype = ctypes.c_int
    lib.aec_crn_last_error.argtypes = [P]
    lib.aec_crn_last_error.restype = ctypes.c_char_p
    lib.aec_crn_destroy.argtypes = [P]
    lib.aec_crn_destroy.restype = None
    _lib = lib
    return lib


def build_info():
    """aec_build_info(): dict(arch, ab_knobs (bool), mode_knobs (list of names))."""
    lib = load()
    if not hasattr(lib, 'aec_build_info'):     # an older A/B build (AEC_HIP_LIB)
        return dict(arch=None, ab_knobs=True, mode_knobs=[], text='(no aec_build_info: older build)')
    txt = lib.aec_build_info().decode()
    head, _, knobs = txt.partition(' mode_knobs=')
    d = dict(kv.split('=', 1) for kv in head.split())
    return dict(arch=d.get('arch'), ab_knobs=d.get('ab_knobs') == 'on',
                mode_knobs=[k.split('(')[0] for k in knobs.split()], text=txt)


def check(status, handle=None, what='', crn=False):
    if status == AEC_OK:
        return
    msg = ''
    if handle is not None and _lib is not None:
        m = (_lib.aec_crn_last_error if crn else _lib.aec_last_error)(handle)
        msg = m.decode() if m else ''
    raise RuntimeError(f'{what} failed: {_STATUS.get(status, status)} {msg}'.strip())


def erb_tables_check(erb, mags, est):
    """Host-side application of the device ERB tables (include/aec_hip.h)."""
    import numpy as np
    lib = load()
    erb = np.ascontiguousarray(erb, np.float32)
    mags = np.ascontiguousarray(mags, np.float32)
    est = np.ascontiguousarray(est, np.float32)
    bands = np.zeros(32, np.float32)
    gains = np.zeros(257, np.float32)
    L = ctypes.c_int32()
    nc = ctypes.c_int32()
    check(lib.aec_erb_tables_check(erb.ctypes.data, mags.ctypes.data, est.ctypes.data, bands.ctypes.data,
                                   gains.ctypes.data, ctypes.byref(L), ctypes.byref(nc)), None,
          'aec_erb_tables_check')
    return bands, gains, int(L.value), int(nc.value)


class Handle:
    """Owns one aec_handle (one per device)."""

    def __init__(self, device: int, nlms_taps=0, nlms_mu=0.5, nlms_beta=0.9, nlms_delta=1e-4):
        self.lib = load()
        cfg = AecConfig(512, 256, 32, int(nlms_taps), float(nlms_mu), float(nlms_beta), float(nlms_delta), 0)
        h = ctypes.c_void_p()
        st = self.lib.aec_create(ctypes.byref(cfg), None, 0, None, int(device), ctypes.byref(h))
        check(st, None, 'aec_create')
        self.h = h
        self.device = device

    def set_weights(self, blob):
        import numpy as np
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        check(self.lib.aec_set_weights(self.h, blob.ctypes.data, blob.size), self.h, 'aec_set_weights')

    def set_erb(self, erb):
        import numpy as np
        erb = np.ascontiguousarray(erb, dtype=np.float32)
        if erb.shape != (257, 32):
            raise ValueError(f'erb must be [257, 32], got {tuple(erb.shape)}')
        check(self.lib.aec_set_erb(self.h, erb.ctypes.data), self.h, 'aec_set_erb')

    def set_debug(self, on: bool):
        check(self.lib.aec_set_debug(self.h, int(bool(on))), self.h, 'aec_set_debug')

    def process(self, mic_ptr, ref_ptr, near_ptr, lengths, B, ld, out_ptr, ld_out, loss_ptr, stream, token=0):
        """lengths: [B] (one length per stream) or [B, 3] (mic, ref, near lengths:
        aec_process_siglens); token: a look-ahead of prepare() to consume
        (aec_process_prepared), 0 = none."""
        import numpy as np
        lens = np.ascontiguousarray(lengths, dtype=np.int64)
        if token:
            if lens.ndim == 1:
                lens = np.repeat(lens[:, None], 3, axis=1)
            st = self.lib.aec_process_prepared(self.h, int(token), mic_ptr, ref_ptr, near_ptr, lens.ctypes.data, int(B),
                                               int(ld), out_ptr, int(ld_out), loss_ptr, stream)
            check(st, self.h, 'aec_process_prepared')
            return
        fn = self.lib.aec_process_siglens if lens.ndim == 2 else self.lib.aec_process
        st = fn(self.h, mic_ptr, ref_ptr, near_ptr, lens.ctypes.data, int(B), int(ld),
                out_ptr, int(ld_out), loss_ptr, stream)
        check(st, self.h, 'aec_process_siglens' if lens.ndim == 2 else 'aec_process')

    def prepare(self, mic_ptr, ref_ptr, near_ptr, lengths, B, ld, stream):
        """Look-ahead normaliser pass of the batch a later process(token=...) takes
        (aec_prepare[_siglens]); returns its token."""
        import numpy as np
        lens = np.ascontiguousarray(lengths, dtype=np.int64)
        fn = self.lib.aec_prepare_siglens if lens.ndim == 2 else self.lib.aec_prepare
        tok = ctypes.c_uint64(0)
        st = fn(self.h, mic_ptr, ref_ptr, near_ptr, lens.ctypes.data, int(B), int(ld), stream, ctypes.byref(tok))
        check(st, self.h, 'aec_prepare_siglens' if lens.ndim == 2 else 'aec_prepare')
        return int(tok.value)

    def stream_open(self, B):
        check(self.lib.aec_stream_open(self.h, int(B)), self.h, 'aec_stream_open')

    def stream_reset(self, b, stream):
        check(self.lib.aec_stream_reset(self.h, int(b), stream), self.h, 'aec_stream_reset')

    def stream_step(self, mic_ptr, ref_ptr, ld_in, out_ptr, ld_out, stream):
        check(self.lib.aec_stream_step(self.h, mic_ptr, ref_ptr, int(ld_in), out_ptr, int(ld_out), stream), self.h,
              'aec_stream_step')

    def debug_copy(self, what, dst_ptr, n, stream):
        check(self.lib.aec_debug_copy(self.h, int(what), dst_ptr, int(n), stream), self.h, 'aec_debug_copy')

    def profile_enable(self, on: bool):
        check(self.lib.aec_profile_enable(self.h, int(bool(on))), self.h, 'aec_profile_enable')

    def profile_read(self):
        """-> (ms per kernel [moments, analysis, gru, synthesis] summed, calls)"""
        ms = (ctypes.c_double * 4)()
        calls = ctypes.c_int64()
        check(self.lib.aec_profile_read(self.h, ms, ctypes.byref(calls)), self.h, 'aec_profile_read')
        return list(ms), int(calls.value)

    # --- training (include/aec_hip.h aec_train_*) --------------------------------
    def set_weights_device(self, ptr, n, stream):
        check(self.lib.aec_set_weights_device(self.h, ptr, int(n), stream), self.h, 'aec_set_weights_device')

    def train_forward(self, mic_ptr, ref_ptr, near_ptr, n, B, ld, out_ptr, ld_out, loss_ptr, stream):
        check(self.lib.aec_train_forward(self.h, mic_ptr, ref_ptr, near_ptr, int(n), int(B), int(ld), out_ptr,
                                         int(ld_out), loss_ptr, stream), self.h, 'aec_train_forward')

    def train_backward(self, grad_loss_ptr, grad_ptr, stream):
        check(self.lib.aec_train_backward(self.h, grad_loss_ptr, grad_ptr, stream), self.h, 'aec_train_backward')

    def train_generation(self):
        return int(self.lib.aec_train_generation(self.h))

    def adam_step(self, p_ptr, g_ptr, m_ptr, v_ptr, n, step, lr, beta1, beta2, eps, weight_decay, stream):
        check(self.lib.aec_adam_step(self.h, p_ptr, g_ptr, m_ptr, v_ptr, int(n), int(step), float(lr), float(beta1),
                                     float(beta2), float(eps), float(weight_decay), stream), self.h, 'aec_adam_step')

    def adam_step_multi(self, p_ptrs, g_ptrs, m_ptrs, v_ptrs, sizes, steps, lr, beta1, beta2, eps, weight_decay,
                        stream):
        n = len(p_ptrs)
        arr = lambda xs: (ctypes.c_void_p * max(n, 1))(*xs)
        i64 = lambda xs: (ctypes.c_int64 * max(n, 1))(*[int(x) for x in xs])
        check(self.lib.aec_adam_step_multi(self.h, arr(p_ptrs), arr(g_ptrs), arr(m_ptrs), arr(v_ptrs), i64(sizes),
                                           i64(steps), n, float(lr), float(beta1), float(beta2), float(eps),
                                           float(weight_decay), stream), self.h, 'aec_adam_step_multi')

    def __del__(self):
        try:
            if getattr(self, 'h', None):
                self.lib.aec_destroy(self.h)
                self.h = None
        except Exception:
            pass


def crn_config(version, conf, dtype, nlms=None):
    """aec_crn_config from a reference config dict (configs.net_conf, configs.py:29-46);
    nlms: None (the reference network) or dict(taps, mu, beta, delta) for the
    build-defined FD-NLMS front end (include/aec_crn.h)."""
    ch = list(conf['conv_channels'])
    if len(ch) > 9:
        raise NotImplementedError('at most 8 encoder layers')
    c = CrnConfig()
    c.version = int(version)
    c.n_layers = len(ch) - 1
    for i, v in enumerate(ch):
        c.conv_channels[i] = int(v)
    c.hidden_dim = int(conf.get('hidden_dim', 4))
    c.rnn_layers = int(conf.get('rnn_layers', 1))
    c.use_cbn = int(bool(conf.get('use_cbn', False)))
    c.masking_mode = ord(conf.get('masking_mode', 'C')[0]) if version == 2 else ord('C')
    c.dtype = {'f32': 0, 'float32': 0, 'bf16': 1, 'bfloat16': 1, 'fp8': 2, 'mxfp8': 2}[dtype]
    if nlms:
        c.nlms_taps = int(nlms.get('taps', 4))
        c.nlms_mu = float(nlms.get('mu', 0.3))
        c.nlms_beta = float(nlms.get('beta', 0.5))
        c.nlms_delta = float(nlms.get('delta', 1e-4))
    return c


def crn_param_count(version, conf, dtype='f32'):
    cfg = crn_config(version, conf, dtype)
    return int(load().aec_crn_param_count(ctypes.byref(cfg)))


class CrnHandle:
    """Owns one aec_crn_handle (include/aec_crn.h), one per device."""

    def __init__(self, version, conf, dtype, device: int, nlms=None):
        self.lib = load()
        self.cfg = crn_config(version, conf, dtype, nlms)
        h = ctypes.c_void_p()
        check(self.lib.aec_crn_create(ctypes.byref(self.cfg), None, 0, int(device), ctypes.byref(h)), None,
              'aec_crn_create (unsupported config?)')
        self.h = h
        self.device = device

    def set_params(self, blob):
        import numpy as np
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        check(self.lib.aec_crn_set_params(self.h, blob.ctypes.data, blob.size), self.h, 'aec_crn_set_params', True)

    def process(self, mic_ptr, far_ptr, lengths, B, ld, out_ptr, ld_out, spec_ptr, mask_ptr, stream):
        import numpy as np
        lens = np.ascontiguousarray(lengths, dtype=np.int64)
        check(self.lib.aec_crn_process(self.h, mic_ptr, far_ptr, lens.ctypes.data, int(B), int(ld), out_ptr,
                                       int(ld_out), spec_ptr, mask_ptr, stream), self.h, 'aec_crn_process', True)

    def stft(self, x_ptr, lengths, B, ld, spec_ptr, stream):
        import numpy as np
        lens = np.ascontiguousarray(lengths, dtype=np.int64)
        check(self.lib.aec_crn_stft(self.h, x_ptr, lens.ctypes.data, int(B), int(ld), spec_ptr, stream), self.h,
              'aec_crn_stft', True)

    def error_spec(self, spec_ptr, stream):
        check(self.lib.aec_crn_error_spec(self.h, spec_ptr, stream), self.h, 'aec_crn_error_spec', True)

    def stream_open(self, B):
        check(self.lib.aec_crn_stream_open(self.h, int(B)), self.h, 'aec_crn_stream_open', True)

    def stream_reset(self, b, stream):
        check(self.lib.aec_crn_stream_reset(self.h, int(b), stream), self.h, 'aec_crn_stream_reset', True)

    def stream_step(self, mic_ptr, far_ptr, ld_in, out_ptr, ld_out, stream):
        check(self.lib.aec_crn_stream_step(self.h, mic_ptr, far_ptr, int(ld_in), out_ptr, int(ld_out), stream),
              self.h, 'aec_crn_stream_step', True)

    def stream_set_graph(self, mode):
        check(self.lib.aec_crn_stream_set_graph(self.h, int(mode)), self.h, 'aec_crn_stream_set_graph', True)

    def stream_stats(self):
        """-> dict(graph_mode, graph_replays, direct_hops) of the open streams"""
        m, g, d = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.aec_crn_stream_stats(self.h, ctypes.byref(m), ctypes.byref(g), ctypes.byref(d)), self.h,
              'aec_crn_stream_stats', True)
        return dict(graph_mode=int(m.value), graph_replays=int(g.value), direct_hops=int(d.value))

    def profile_enable(self, on: bool):
        check(self.lib.aec_crn_profile_enable(self.h, int(bool(on))), self.h, 'aec_crn_profile_enable', True)

    def profile_read(self):
        """-> (ms [front, encoder, lstm, decoder, back] summed, calls)"""
        ms = (ctypes.c_double * 5)()
        calls = ctypes.c_int64()
        check(self.lib.aec_crn_profile_read(self.h, ms, ctypes.byref(calls)), self.h, 'aec_crn_profile_read', True)
        return list(ms), int(calls.value)

    def __del__(self):
        try:
            if getattr(self, 'h', None):
                self.lib.aec_crn_destroy(self.h)
                self.h = None
        except Exception:
            pass

