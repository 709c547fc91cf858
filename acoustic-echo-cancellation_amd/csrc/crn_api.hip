// crn_api.hip — the DCCRN C ABI (include/aec_crn.h) over crn_kernels.hip.
//
// Host side of the reference's DCCRN eval forward (Stage2_lhm/scripts/
// network/dccrn.py:453-594, dccrn2.py:10-218): parses the state_dict-ordered
// parameter blob, folds every eval-mode BatchNorm2d / ComplexBatchNorm into
// its complex conv (float64), permutes weights into the kernels' layouts
// (channels-last maps, decoder skip order, LSTM unit order and gate packing),
// owns a grow-only workspace and sequences the launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <cstdio>
#include <vector>

#include "../../include/aec_crn.h"
#include "aec_device.h"
#include "aec_launch.h"
#include "aec_tables.h"
#include "crn_launch.h"

using crn::bf16_t;

namespace {

int ilog2(int64_t v) {
    int r = 0;
    while ((1ll << r) < v) ++r;
    return (1ll << r) == v ? r : -1;
}

uint16_t host_f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)(u >> 16) | ((u & 0xFFFF) ? 0x40 : 0);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

struct Cursor {
    const float* p;
    size_t n, off = 0;
    bool ok = true;
    const float* take(size_t k) {
        if (off + k > n) {
            ok = false;
            return nullptr;
        }
        const float* r = p + off;
        off += k;
        return r;
    }
};

// A packed GEMM weight operand (device) + bias
struct Packed {
    void* w = nullptr;          // [npad][kpad] elements of the compute type
    float* bias = nullptr;      // [npad]
    int npad = 0, kpad = 0, N = 0, K = 0;
    float alpha = 0.f;
    int act = 0;
    uint8_t* wq = nullptr;      // dtype 2 (LSTM input projections, qualifying conv layers): e4m3 [npad8][kpad]
    uint8_t* wsc = nullptr;     //   and E8M0 scales [npad8][kpad / 32]
    int npad8 = 0;              // rows of wq (a multiple of the MX GEMM's 256-column tile)
};

}  // namespace

struct StreamState;

struct aec_crn_handle {
    aec_crn_config cfg{};
    int device = 0;
    std::string err;
    int L = 6, D = 4, H = 0, S = 1, CELLS = 1, Q = 0, nrnn = 1;
    size_t es = 4;                                 // element size
    bool mx8 = false;                              // dtype 2: MX-fp8 LSTM input projections
    aec::DevTables* d_tab = nullptr;
    std::vector<Packed> enc, dec;                  // dec: 2 per level (even, odd)
    std::vector<Packed> decf;                      // per level: both parities in one GEMM (see pack_decoder_fused)
    int dec_fuse_max = 128;                        // CRN_DEC_FUSE: fuse the parities of levels with <= this many
                                                   // output channels (HBM-bound layers); 0 = never
    std::vector<Packed> lih, lhh;                  // per LSTM layer
    std::vector<Packed> lcat;                      // dtype 2, v2: [W_ih | W_hh] MX rows (lstm_step_mx8_kernel)
    bool have_params = false;
    // workspace
    int64_t ws_B = 0, ws_T = 0;
    void* x0 = nullptr;
    std::vector<void*> cat;                        // index 1..L
    void* gx = nullptr;
    void* y = nullptr;
    void* xn = nullptr;
    uint8_t* aq = nullptr;                         // dtype 2: quantized rows + scales (layers without a shadow)
    uint8_t* as = nullptr;
    bool mx8_shadow = true;                        // AEC_CRN_MX8_SHADOW=0 at create: every MX GEMM quantises its rows
                                                   //   first (the A/B and bit-equality reference)
    std::vector<uint8_t*> cat8, cats;              // dtype 2: MX-fp8 shadows of cat[l] (null: none), see shadow_level
    uint8_t* xn8 = nullptr;                        //   and of xn
    uint8_t* xns = nullptr;
    float* cst = nullptr;
    float* mask = nullptr;
    float2* nrows = nullptr;                       // NLMS: packed mic / far rows [B][T][2][256]
    float2* espec = nullptr;                       //       error rows E [B][T][256]
    float2* ndummy = nullptr;                      //       [B][256] sink for frames past a stream's end
    int64_t* d_len = nullptr;
    std::vector<int64_t> last_lens;                // host copy of what d_len holds
    int32_t last_B = 0;                            // shape of the last aec_crn_process call (aec_crn_error_spec)
    int64_t last_T = 0;
    std::vector<int64_t> proc_lens;                //   and its lengths
    std::vector<void*> allocs;
    StreamState* ss = nullptr;                     // aec_crn_stream_* state
    // persistent LSTM recurrence (crn_persist.hip; AEC_CRN_PERSIST=0: one launch per frame)
    int persist = 1;
    int num_cus = 0;
    int* psync = nullptr;                          // arrival counters + error word
    int* perr_host = nullptr;                      // pinned copy of the error word, read back per call
    hipEvent_t perr_ev = nullptr;                  // recorded after that copy
    int persist_timeouts = 0;                      // consecutive calls that timed out (2: persist = 0)
    bool persist_pending = false;                  // this call launched persistent grids: check before returning
    // profiling
    int profile = 0;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    double ms[5] = {0, 0, 0, 0, 0};
    int64_t calls = 0;
};

#define CRN_TRY(h, expr)                                                                 \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            (h)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                \
            return e_ == hipErrorOutOfMemory ? AEC_ERR_OOM : AEC_ERR_HIP;                \
        }                                                                                \
    } while (0)

static aec_status crn_fail(aec_crn_handle* h, aec_status s, const std::string& m) {
    if (h) h->err = m;
    return s;
}

// --------------------------------------------------------------------------
// config validation + parameter layout
// --------------------------------------------------------------------------
static std::string check_cfg(const aec_crn_config& c) {
    if (c.version != 1 && c.version != 2) return "version must be 1 (dccrn.py) or 2 (dccrn2.py)";
    if (c.n_layers < 1 || c.n_layers > 8) return "n_layers out of range";
    if (256 >> c.n_layers != 4) return "the LSTM width needs 256 >> n_layers == 4 (dccrn.py:514)";
    if (c.conv_channels[0] != 4) return "conv_channels[0] must be 4 (mic/far real/imag)";
    for (int i = 1; i <= c.n_layers; ++i)
        if (c.conv_channels[i] < 8 || ilog2(c.conv_channels[i]) < 0) return "conv_channels must be powers of two >= 8";
    if (c.dtype < 0 || c.dtype > 2) return "dtype must be 0 (f32), 1 (bf16) or 2 (bf16 + MX-fp8 LSTM input)";
    if (c.version == 2) {
        if (c.hidden_dim != 4) return "hidden_dim must equal the encoder output width (4)";
        if (c.rnn_layers < 1 || c.rnn_layers > 8) return "rnn_layers out of range";
        if (c.masking_mode != 'E' && c.masking_mode != 'C' && c.masking_mode != 'R') return "masking_mode must be E, C or R";
    }
    if (c.nlms_taps < 0 || c.nlms_taps > 8) return "nlms_taps must be 0..8";
    if (c.nlms_taps > 0 && !(c.nlms_mu >= 0.f && c.nlms_mu < 2.f && c.nlms_beta >= 0.f && c.nlms_beta < 1.f &&
                             c.nlms_delta > 0.f))
        return "NLMS needs mu in [0, 2), beta in [0, 1), delta > 0";
    return "";
}

static size_t norm_count(const aec_crn_config& c, int ch) {
    return (c.version == 2 && c.use_cbn) ? 10 * (size_t)(ch / 2) : 4 * (size_t)ch;
}

static size_t param_count(const aec_crn_config& c) {
    if (!check_cfg(c).empty()) return 0;
    const int* ch = c.conv_channels;
    const int L = c.n_layers;
    size_t n = 0;
    for (int i = 0; i < L; ++i) {
        const size_t co = ch[i + 1] / 2, ci = ch[i] / 2;
        n += 2 * (co * ci * 5 + co) + norm_count(c, ch[i + 1]) + 1;
    }
    for (int cl = L; cl >= 1; --cl) {
        const size_t ci = ch[cl], co = (cl != 1 ? ch[cl - 1] : 2) / 2;
        n += 2 * (ci * co * 5 + co);
        if (cl != 1)
            n += norm_count(c, ch[cl - 1]) + 1;
        else if (c.version == 1)
            n += 4 * 2;
    }
    if (c.version == 1) {
        const size_t H = (size_t)ch[L] * 4;
        n += 2 * 4 * H * H + 2 * 4 * H;
    } else {
        const size_t H = (size_t)c.hidden_dim * ch[L] / 2;
        n += (size_t)c.rnn_layers * 2 * (2 * 4 * H * H + 2 * 4 * H);
    }
    return n;
}

// --------------------------------------------------------------------------
// folding: complex conv -> real [Co][Ci][5] (out x in, reference channel
// order) + bias; then the eval norm as an affine map on the output channels
// --------------------------------------------------------------------------
struct RealConv {
    int Co = 0, Ci = 0;
    std::vector<double> w;   // [Co][Ci][5]
    std::vector<double> b;   // [Co]
    double& at(int o, int i, int k) { return w[((size_t)o * Ci + i) * 5 + k]; }
};

// ComplexConv2d (dccrn.py:140-153): weights [co'][ci'][5][1];
// ComplexConvTranspose2d (dccrn.py:194-207): weights [ci'][co'][5][1].
static RealConv complex_conv(Cursor& cur, int Ci, int Co, bool transposed) {
    const int ci = Ci / 2, co = Co / 2;
    const size_t nw = (size_t)ci * co * 5;
    const float* wr = cur.take(nw);
    const float* br = cur.take(co);
    const float* wi = cur.take(nw);
    const float* bi = cur.take(co);
    RealConv r;
    r.Co = Co;
    r.Ci = Ci;
    r.w.assign((size_t)Co * Ci * 5, 0.0);
    r.b.assign(Co, 0.0);
    if (!cur.ok) return r;
    for (int o = 0; o < co; ++o)
        for (int i = 0; i < ci; ++i)
            for (int k = 0; k < 5; ++k) {
                const size_t idx = transposed ? ((size_t)i * co + o) * 5 + k : ((size_t)o * ci + i) * 5 + k;
                const double a = wr[idx], c = wi[idx];
                r.at(o, i, k) = a;            // real <- real_conv(x_r)
                r.at(o, ci + i, k) = -c;      //       - imag_conv(x_i)
                r.at(co + o, i, k) = c;       // imag <- imag_conv(x_r)
                r.at(co + o, ci + i, k) = a;  //       + real_conv(x_i)
            }
    for (int o = 0; o < co; ++o) {
        r.b[o] = (double)br[o] - (double)bi[o];
        r.b[co + o] = (double)bi[o] + (double)br[o];
    }
    return r;
}

// y = A z + c0 per output channel (pairs (o, co+o) for ComplexBatchNorm)
static void fold_norm(Cursor& cur, RealConv& r, bool cbn) {
    const int Co = r.Co;
    const double eps = 1e-5;
    std::vector<double> A((size_t)Co * Co, 0.0), c0(Co, 0.0);
    if (cbn) {   // ComplexBatchNorm eval (dccrn.py:300-383)
        const int c = Co / 2;
        const float *Wrr = cur.take(c), *Wri = cur.take(c), *Wii = cur.take(c), *Br = cur.take(c), *Bi = cur.take(c);
        const float *RMr = cur.take(c), *RMi = cur.take(c), *RVrr = cur.take(c), *RVri = cur.take(c),
                    *RVii = cur.take(c);
        if (!cur.ok) return;
        for (int o = 0; o < c; ++o) {
            const double Vrr = (double)RVrr[o] + eps, Vri = RVri[o], Vii = (double)RVii[o] + eps;
            const double tau = Vrr + Vii;
            const double s = std::sqrt(Vrr * Vii - Vri * Vri);
            const double t = std::sqrt(tau + 2 * s);
            const double rst = 1.0 / (s * t);
            const double Urr = (s + Vii) * rst, Uii = (s + Vrr) * rst, Uri = -Vri * rst;
            const double Zrr = Wrr[o] * Urr + Wri[o] * Uri;
            const double Zri = Wrr[o] * Uri + Wri[o] * Uii;
            const double Zir = Wri[o] * Urr + Wii[o] * Uri;
            const double Zii = Wri[o] * Uri + Wii[o] * Uii;
            A[(size_t)o * Co + o] = Zrr;
            A[(size_t)o * Co + c + o] = Zri;
            A[(size_t)(c + o) * Co + o] = Zir;
            A[(size_t)(c + o) * Co + c + o] = Zii;
            c0[o] = Br[o] - Zrr * RMr[o] - Zri * RMi[o];
            c0[c + o] = Bi[o] - Zir * RMr[o] - Zii * RMi[o];
        }
    } else {     // BatchNorm2d eval
        const float *w = cur.take(Co), *b = cur.take(Co), *rm = cur.take(Co), *rv = cur.take(Co);
        if (!cur.ok) return;
        for (int o = 0; o < Co; ++o) {
            const double s = (double)w[o] / std::sqrt((double)rv[o] + eps);
            A[(size_t)o * Co + o] = s;
            c0[o] = (double)b[o] - s * rm[o];
        }
    }
    RealConv f = r;
    for (int o = 0; o < Co; ++o) {
        for (size_t q = 0; q < (size_t)r.Ci * 5; ++q) {
            double acc = 0;
            for (int o2 = 0; o2 < Co; ++o2) {
                const double a = A[(size_t)o * Co + o2];
                if (a != 0.0) acc += a * r.w[(size_t)o2 * r.Ci * 5 + q];
            }
            f.w[(size_t)o * r.Ci * 5 + q] = acc;
        }
        double acc = c0[o];
        for (int o2 = 0; o2 < Co; ++o2) acc += A[(size_t)o * Co + o2] * r.b[o2];
        f.b[o] = acc;
    }
    r = f;
}

static aec_status upload_packed(aec_crn_handle* h, Packed& pk, const std::vector<double>& w,
                                const std::vector<double>& b) {
    const size_t n = (size_t)pk.npad * pk.kpad;
    if (!pk.w) {
        CRN_TRY(h, hipMalloc(&pk.w, n * h->es));
        CRN_TRY(h, hipMalloc(&pk.bias, (size_t)pk.npad * sizeof(float)));
    }
    if (h->es == 4) {
        std::vector<float> hw(n);
        for (size_t i = 0; i < n; ++i) hw[i] = (float)w[i];
        CRN_TRY(h, hipMemcpy(pk.w, hw.data(), n * 4, hipMemcpyHostToDevice));
    } else {
        std::vector<uint16_t> hw(n);
        for (size_t i = 0; i < n; ++i) hw[i] = host_f2bf((float)w[i]);
        CRN_TRY(h, hipMemcpy(pk.w, hw.data(), n * 2, hipMemcpyHostToDevice));
    }
    std::vector<float> hb(pk.npad, 0.f);
    for (int i = 0; i < pk.N; ++i) hb[i] = (float)b[i];
    CRN_TRY(h, hipMemcpy(pk.bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    return AEC_OK;
}

// OCP e4m3 (e4m3fn) of x, round to nearest even, saturating at +-448
static uint8_t host_e4m3(double x) {
    const uint8_t sg = x < 0 ? 0x80 : 0;
    const double a = std::fabs(x);
    if (!(a < 448.0)) return sg | 0x7E;
    if (a < std::ldexp(1.0, -6)) return sg | (uint8_t)std::nearbyint(a * 512.0);   // subnormal: m * 2^-9
    int e2;
    (void)std::frexp(a, &e2);
    const int E = e2 - 1;                                                          // floor(log2 a), -6 .. 8
    const int m = (int)std::nearbyint((a / std::ldexp(1.0, E) - 1.0) * 8.0);      // 0 .. 8 (8 carries)
    const int code = std::min(((E + 7) << 3) + m, 0x7E);
    return sg | (uint8_t)code;
}

// dtype 2: the packed weight rows [npad][kpad] as MX-fp8 (E8M0 scale per 32 k:
// 2^(floor(log2 amax) - 8), the same rule as the device's activation quantizer)
static aec_status upload_mx8(aec_crn_handle* h, Packed& pk, const std::vector<double>& w) {
    pk.npad8 = (pk.N + 255) / 256 * 256;
    const size_t n = (size_t)pk.npad8 * pk.kpad, kb = (size_t)pk.kpad / 32;
    std::vector<uint8_t> q(n, 0), sc((size_t)pk.npad8 * kb, 0);
    for (int r = 0; r < pk.N; ++r)
        for (size_t b = 0; b < kb; ++b) {
            const double* x = &w[(size_t)r * pk.kpad + b * 32];
            double amax = 0;
            for (int j = 0; j < 32; ++j) amax = std::max(amax, std::fabs((double)(float)x[j]));
            int code = 0;
            if (amax > 0) {
                int e2;
                (void)std::frexp((double)(float)amax, &e2);
                code = std::max(0, std::min(254, (e2 - 1) + 127 - 8));
            }
            sc[(size_t)r * kb + b] = (uint8_t)code;
            for (int j = 0; j < 32; ++j)
                q[(size_t)r * pk.kpad + b * 32 + j] = host_e4m3(std::ldexp((double)(float)x[j], 127 - code));
        }
    if (!pk.wq) {
        CRN_TRY(h, hipMalloc(&pk.wq, n));
        CRN_TRY(h, hipMalloc(&pk.wsc, sc.size()));
    }
    CRN_TRY(h, hipMemcpy(pk.wq, q.data(), n, hipMemcpyHostToDevice));
    CRN_TRY(h, hipMemcpy(pk.wsc, sc.data(), sc.size(), hipMemcpyHostToDevice));
    return AEC_OK;
}

// dtype 2 also runs a conv layer on the MX-fp8 GEMM when its implicit rows
// split into 32-k blocks inside one tap (2^kshift % 32 == 0), K is a whole
// number of 128-k stages and the layer is wide enough (N >= 128) for the
// 256-column MX tile: encoder layers 4-5 and decoder levels 5-6 of net_conf,
// about 75 % of the conv FLOPs.
static bool conv_mx8(const aec_crn_handle* h, const Packed& pk, int kshift_ch) {
    return h->mx8 && pk.K % 128 == 0 && pk.kpad == pk.K && kshift_ch % 32 == 0 && pk.N >= 128;
}

static int kpad_for(int K, size_t es) {
    const int per = (int)(crn::kStageBytes / es);
    return (K + per - 1) / per * per;
}

// encoder layer: Bt[co][tap*Cin_buf + q] = W[co][q][tap]  (q < real input channels)
static aec_status pack_encoder(aec_crn_handle* h, Packed& pk, const RealConv& r, int cin_buf, float alpha) {
    pk.N = r.Co;
    pk.K = 5 * cin_buf;
    pk.npad = (r.Co + crn::gemm_bn(r.Co) - 1) / crn::gemm_bn(r.Co) * crn::gemm_bn(r.Co);
    pk.kpad = kpad_for(pk.K, h->es);
    pk.alpha = alpha;
    pk.act = 1;
    std::vector<double> w((size_t)pk.npad * pk.kpad, 0.0);
    for (int o = 0; o < r.Co; ++o)
        for (int k = 0; k < 5; ++k)
            for (int q = 0; q < std::min(cin_buf, r.Ci); ++q)
                w[(size_t)o * pk.kpad + k * cin_buf + q] = r.w[((size_t)o * r.Ci + q) * 5 + k];
    aec_status s = upload_packed(h, pk, w, r.b);
    if (s == AEC_OK && conv_mx8(h, pk, cin_buf)) s = upload_mx8(h, pk, w);
    return s;
}

// decoder level: input buffer channels [dec_r, dec_i, enc_r, enc_i] (C each
// half-pair) vs the reference complex_cat order [dec_r, enc_r, dec_i, enc_i]
// (dccrn.py:386-395); parity 0: taps (4, 2, 0) at bins (m-1, m, m+1),
// parity 1: taps (3, 1) at (m, m+1).
static aec_status pack_decoder(aec_crn_handle* h, Packed& pk, const RealConv& r, int parity, int act, float alpha) {
    const int Cin = r.Ci, C = Cin / 2;
    const int ntap = parity == 0 ? 3 : 2;
    pk.N = r.Co;
    pk.K = ntap * Cin;
    const int bn = crn::gemm_bn(r.Co);
    pk.npad = (r.Co + bn - 1) / bn * bn;
    pk.kpad = kpad_for(pk.K, h->es);
    pk.alpha = alpha;
    pk.act = act;
    auto ref = [&](int q) {
        if (q < C / 2) return q;
        if (q < C) return C + (q - C / 2);
        if (q < 3 * C / 2) return C / 2 + (q - C);
        return q;
    };
    std::vector<double> w((size_t)pk.npad * pk.kpad, 0.0);
    for (int o = 0; o < r.Co; ++o)
        for (int j = 0; j < ntap; ++j) {
            const int tap = parity == 0 ? 4 - 2 * j : 3 - 2 * j;
            for (int q = 0; q < Cin; ++q)
                w[(size_t)o * pk.kpad + j * Cin + q] = r.w[((size_t)o * Cin + ref(q)) * 5 + tap];
        }
    aec_status s = upload_packed(h, pk, w, r.b);
    if (s == AEC_OK && act == 1 && conv_mx8(h, pk, Cin)) s = upload_mx8(h, pk, w);
    return s;
}

// Both parities of a decoder level as ONE GEMM over the rows of parity 0
// (bins m-1, m, m+1): columns [0, Co) parity 0 (taps 4, 2, 0), columns
// [Co, 2 Co) parity 1 (zero at bin m-1, taps 3, 1 at m, m+1).  The
// memory-bound levels read their input rows once instead of twice; the
// epilogue routes the parity-1 columns to the odd output bins (RowEpi nsplit).
static aec_status pack_decoder_fused(aec_crn_handle* h, Packed& pk, const RealConv& r, int act, float alpha) {
    const int Cin = r.Ci, C = Cin / 2, Co = r.Co;
    pk.N = 2 * Co;
    pk.K = 3 * Cin;
    const int bn = crn::gemm_bn(pk.N);
    pk.npad = (pk.N + bn - 1) / bn * bn;
    pk.kpad = kpad_for(pk.K, h->es);
    pk.alpha = alpha;
    pk.act = act;
    auto ref = [&](int q) {
        if (q < C / 2) return q;
        if (q < C) return C + (q - C / 2);
        if (q < 3 * C / 2) return C / 2 + (q - C);
        return q;
    };
    std::vector<double> w((size_t)pk.npad * pk.kpad, 0.0), b(pk.N);
    for (int o = 0; o < Co; ++o) {
        b[o] = b[Co + o] = r.b[o];
        for (int j = 0; j < 3; ++j)
            for (int q = 0; q < Cin; ++q) {
                w[(size_t)o * pk.kpad + j * Cin + q] = r.w[((size_t)o * Cin + ref(q)) * 5 + (4 - 2 * j)];
                if (j > 0) w[(size_t)(Co + o) * pk.kpad + j * Cin + q] = r.w[((size_t)o * Cin + ref(q)) * 5 + (5 - 2 * j)];
            }
    }
    aec_status s = upload_packed(h, pk, w, b);
    // dtype 2: the wide levels on the MX GEMM (parity 1's zero tap is a whole number of 128-k
    // stages, so each parity's sum is the unfused GEMM's, bit for bit)
    if (s == AEC_OK && act == 1 && conv_mx8(h, pk, Cin)) s = upload_mx8(h, pk, w);
    return s;
}

// LSTM cell(s): unit order u' = d*Q + c <-> reference u = c*D + d; W_hh gate
// row p(q, u') = ((u'/16)*4 + q)*16 + u'%16 (i|f|g|o per 16 units), W_ih /
// bias gate row u'*4 + q (so Gx holds a unit's 4 gates contiguously)
static aec_status pack_lstm(aec_crn_handle* h, Cursor& cur, Packed& ih, Packed& hh, Packed& cat) {
    const int H = h->H, D = h->D, Q = h->Q, C = h->CELLS;
    const size_t G = (size_t)4 * H;
    std::vector<double> wih((size_t)C * G * H), whh((size_t)C * G * H), bias((size_t)C * G);
    // dtype 2, NavieComplexLSTM: [W_ih | W_hh] rows (K = 2H) in W_hh's row order for the fused
    // per-hop layer step (lstm_step_mx8_kernel)
    const bool want_cat = h->mx8 && C * h->S == 4 && H % 256 == 0;
    std::vector<double> wcat(want_cat ? (size_t)C * G * 2 * H : 0);
    auto perm = [&](int up) { return (up % Q) * D + up / Q; };
    for (int cell = 0; cell < C; ++cell) {
        const float* Wih = cur.take(G * H);
        const float* Whh = cur.take(G * H);
        const float* bih = cur.take(G);
        const float* bhh = cur.take(G);
        if (!cur.ok) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameter blob too short");
        for (int up = 0; up < H; ++up)
            for (int q = 0; q < 4; ++q) {
                // W_hh rows: fragment order (16 units of one gate per 16-column fragment);
                // W_ih rows / bias: the 4 gates of a unit adjacent (Gx read as one vector)
                const size_t p = (size_t)cell * G + ((size_t)(up / 16) * 4 + q) * 16 + up % 16;
                const size_t pi = (size_t)cell * G + (size_t)up * 4 + q;
                const size_t src = (size_t)q * H + perm(up);
                for (int kp = 0; kp < H; ++kp) {
                    wih[pi * H + kp] = Wih[src * H + perm(kp)];
                    whh[p * H + kp] = Whh[src * H + perm(kp)];
                }
                if (want_cat)
                    for (int kp = 0; kp < H; ++kp) {
                        wcat[p * 2 * H + kp] = Wih[src * H + perm(kp)];
                        wcat[p * 2 * H + H + kp] = Whh[src * H + perm(kp)];
                    }
                bias[pi] = (double)bih[src] + (double)bhh[src];
            }
    }
    ih.N = hh.N = (int)(C * G);
    ih.K = hh.K = H;
    ih.npad = hh.npad = (int)(C * G);
    ih.kpad = hh.kpad = H;
    ih.act = 0;
    aec_status s = upload_packed(h, ih, wih, bias);
    if (s != AEC_OK) return s;
    if (h->mx8) {
        s = upload_mx8(h, ih, wih);
        if (s != AEC_OK) return s;
    }
    s = upload_packed(h, hh, whh, bias);
    if (s == AEC_OK && want_cat) {
        cat.N = (int)(C * G);
        cat.K = cat.kpad = 2 * H;
        s = upload_mx8(h, cat, wcat);
    }
    return s;
}

static aec_status load_params(aec_crn_handle* h, const float* params, size_t n) {
    const aec_crn_config& c = h->cfg;
    if (n != param_count(c)) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameter count mismatch");
    Cursor cur{params, n};
    const int* ch = c.conv_channels;
    const int L = h->L;
    const bool cbn = c.version == 2 && c.use_cbn;
    for (int i = 0; i < L; ++i) {
        RealConv r = complex_conv(cur, ch[i], ch[i + 1], false);
        fold_norm(cur, r, cbn);
        const float* a = cur.take(1);
        if (!cur.ok) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameter blob too short");
        aec_status s = pack_encoder(h, h->enc[i], r, i == 0 ? 8 : ch[i], a[0]);
        if (s != AEC_OK) return s;
    }
    for (int d = 0; d < L; ++d) {
        const int cl = L - d;
        const int co = cl != 1 ? ch[cl - 1] : 2;
        RealConv r = complex_conv(cur, 2 * ch[cl], co, true);
        int act = 0;
        float alpha = 0.f;
        if (cl != 1) {
            fold_norm(cur, r, cbn);
            const float* a = cur.take(1);
            if (!cur.ok) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameter blob too short");
            act = 1;
            alpha = a[0];
        } else if (c.version == 1) {   // BatchNorm2d(2) + Tanh (dccrn.py:494-506)
            fold_norm(cur, r, false);
            act = 2;
        }
        if (!cur.ok) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameter blob too short");
        for (int par = 0; par < 2; ++par) {
            aec_status s = pack_decoder(h, h->dec[2 * d + par], r, par, act, alpha);
            if (s != AEC_OK) return s;
        }
        // fused parities: bf16 / f32 stores of 16 B never straddle the parity
        // split when Co % 8 == 0 (measured, C3 bf16 decoder: unfused 7.31 ms, fused up to
        // Co = 64 6.58, 128 6.42, 256 6.61); with dtype fp8 the levels the MX GEMM takes
        // (Co >= 128) are fused too (one launch per level instead of two in the per-hop step).
        // The mask level (Co = 2, f32 [F][256][2]) is fused as well: the two parities' outputs of
        // an input bin are the 4 adjacent floats of bins 2i, 2i + 1, so its rows need no split
        if ((cl != 1 && co % 8 == 0 && (co <= h->dec_fuse_max || (h->mx8 && h->dec_fuse_max >= 0))) ||
            (cl == 1 && h->dec_fuse_max >= 0)) {
            aec_status s = pack_decoder_fused(h, h->decf[d], r, act, alpha);
            if (s != AEC_OK) return s;
        }
    }
    for (int l = 0; l < h->nrnn; ++l) {
        aec_status s = pack_lstm(h, cur, h->lih[l], h->lhh[l], h->lcat[l]);
        if (s != AEC_OK) return s;
    }
    if (!cur.ok || cur.off != n) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameter blob layout mismatch");
    h->have_params = true;
    return AEC_OK;
}

// dtype 2: bytes per frame of the largest quantized row block (LSTM input
// rows, or the implicit rows of an MX-fp8 conv layer)
static size_t mx8_row_bytes(const aec_crn_handle* h) {
    size_t m = (size_t)h->S * h->H;
    for (int i = 0; i < h->L; ++i)
        if (h->enc[i].wq) m = std::max(m, (size_t)(128 >> i) * h->enc[i].K);
    for (int d = 0; d < h->L; ++d)
        for (int par = 0; par < 2; ++par)
            if (h->dec[2 * d + par].wq) m = std::max(m, (size_t)(256 >> (h->L - d)) * h->dec[2 * d + par].K);
    return m;
}

// dtype 2: cat[l] gets an MX-fp8 shadow (written by every producer's epilogue,
// read in place by the MX GEMMs: no separate quantisation pass) when an MX
// layer consumes it and its rows qualify for the in-place gather (128 | 2^kshift):
// encoder layer l, decoder level l, or the first LSTM layer (l == L)
static bool shadow_level(const aec_crn_handle* h, int l) {
    if (!h->mx8 || !h->mx8_shadow || l < 1 || l > h->L) return false;
    // cat[L]'s dec half comes from the LSTM combine, which writes a shadow for NavieComplexLSTM (v2) only
    if (l == h->L && h->CELLS * h->S != 4) return false;
    const int* ch = h->cfg.conv_channels;
    if (l < h->L && h->enc[l].wq && ch[l] % 128 == 0) return true;
    const int d = h->L - l;
    if ((h->dec[2 * d].wq || h->dec[2 * d + 1].wq) && (2 * ch[l]) % 128 == 0) return true;
    return l == h->L && h->Q % 128 == 0 && (2 * ch[l]) % 128 == 0;
}
static bool shadow_xn(const aec_crn_handle* h) {
    return h->mx8 && h->mx8_shadow && h->nrnn > 1 && h->Q % 128 == 0 && h->CELLS * h->S == 4;
}

static aec_status ensure_ws(aec_crn_handle* h, int64_t B, int64_t T) {
    if (B <= h->ws_B && T <= h->ws_T) return AEC_OK;
    for (void* p : h->allocs) (void)hipFree(p);
    h->allocs.clear();
    h->last_lens.clear();                          // d_len is reallocated below
    h->last_B = 0;                                 // and the NLMS rows with it
    const int64_t nB = std::max<int64_t>(B, h->ws_B), nT = std::max<int64_t>(T, h->ws_T);
    const int64_t BT = nB * nT;
    const size_t es = h->es;
    auto alloc = [&](void** p, size_t bytes) {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
        if (e == hipSuccess) h->allocs.push_back(*p);
        return e;
    };
    const int* ch = h->cfg.conv_channels;
    CRN_TRY(h, alloc(&h->x0, (size_t)BT * 256 * 8 * es));
    h->cat.assign(h->L + 1, nullptr);
    for (int l = 1; l <= h->L; ++l) CRN_TRY(h, alloc(&h->cat[l], (size_t)BT * (256 >> l) * 2 * ch[l] * es));
    CRN_TRY(h, alloc(&h->gx, (size_t)BT * h->S * h->CELLS * 4 * h->H * es));
    CRN_TRY(h, alloc(&h->y, (size_t)BT * h->CELLS * h->S * h->H * es));
    if (h->nrnn > 1) CRN_TRY(h, alloc(&h->xn, (size_t)BT * h->S * h->H * es));
    if (h->mx8) {
        const size_t qb = (size_t)BT * mx8_row_bytes(h);
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->aq), qb));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->as), qb / 32));
    }
    h->cat8.assign(h->L + 1, nullptr);
    h->cats.assign(h->L + 1, nullptr);
    for (int l = 1; l <= h->L; ++l)
        if (shadow_level(h, l)) {
            const size_t n8 = (size_t)BT * (256 >> l) * 2 * ch[l];
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->cat8[l]), n8));
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->cats[l]), n8 / 32));
        }
    h->xn8 = h->xns = nullptr;
    if (shadow_xn(h)) {
        const size_t n8 = (size_t)BT * h->S * h->H;
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->xn8), n8));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->xns), n8 / 32));
    }
    CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->cst), (size_t)nB * h->CELLS * h->S * h->H * sizeof(float)));
    CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->mask), (size_t)BT * 256 * 2 * sizeof(float)));
    CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->d_len), (size_t)nB * sizeof(int64_t)));
    if (h->cfg.nlms_taps > 0) {
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->nrows), (size_t)BT * 512 * sizeof(float2)));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->espec), (size_t)BT * 256 * sizeof(float2)));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&h->ndummy), (size_t)nB * 256 * sizeof(float2)));
    }
    h->ws_B = nB;
    h->ws_T = nT;
    return AEC_OK;
}

static void mark(aec_crn_handle* h, hipStream_t st) {
    if (!h->profile) return;
    if (h->ev_used == h->ev.size()) {
        hipEvent_t e;
        // timing marks without the system-scope release fence a default event adds
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return;
        h->ev.push_back(e);
    }
    (void)hipEventRecord(h->ev[h->ev_used++], st);
}

// Feature buffers of one pass over F frames (batch: F = B*Tmax; stream: F = B)
struct Bufs {
    void* x0;
    void* const* cat;       // [L+1], index 1..L
    void* gx;
    void* xn;
    float* mask;
    uint8_t* aq;            // dtype 2: quantized rows [rows][K] + scales [rows][K/32] (layers without a shadow)
    uint8_t* as;
    uint8_t* const* cat8;   // dtype 2: MX-fp8 shadows of cat[l] (e4m3 [F][bins][2 ch], E8M0 per 32), null: none
    uint8_t* const* cats;
    uint8_t* xn8;           //   and of xn
    uint8_t* xns;
    // split-K workspace of the MX conv GEMMs (per-hop streaming only; null: no split)
    float* skp = nullptr;
    int* skc = nullptr;
    int64_t sk_bytes = 0;
    int32_t skc_n = 0;
};

// K slices of an MX conv GEMM in the per-hop step (its grid alone covers a fraction of the
// CUs): >= 3 stages of 128 k per slice.  Chosen per layer, never from the row count.
static int conv_ksplit(int kpad) {
    static const int mx = AEC_AB_KNOB("AEC_CRN_SPLITK", 4);
    const int nst = kpad / 128;
    int ks = 1;
    while (ks * 2 <= mx && nst >= 6 * ks) ks *= 2;
    return ks;
}

// an output with an MX-fp8 shadow (bf16 GEMM epilogues only)
template <typename T>
static void set_shadow(crn::RowEpi& e, uint8_t* q8, uint8_t* qs) {
    if (sizeof(T) == 2 && q8 && e.N % 128 == 0) {      // the 128-column tiles: 32-column groups in lane quads
        e.q8 = q8;
        e.qs = qs;
    }
}

// dtype 2 GEMM over the implicit rows `a`: in place from the source's MX-fp8 shadow
// (q8 / qs, written by its producers), else quantised into bf.aq / bf.as first
template <typename T>
static aec_status mx8_gemm(aec_crn_handle* h, const crn::RowSrc& a, const uint8_t* q8, const uint8_t* qs,
                           const Bufs& bf, const uint8_t* wq, const uint8_t* wsc, int K, const crn::RowEpi& e0, int npad,
                           hipStream_t st, bool conv = false) {
    crn::RowEpi e = e0;
    if (conv && bf.skp) {
        e.ksplit = conv_ksplit(K);
        e.skp = bf.skp;
        e.skc = bf.skc;
        e.sk_bytes = bf.sk_bytes;
        e.skc_n = bf.skc_n;
    }
    if (q8) {
        crn::RowSrc a8 = a;
        a8.src = q8;
        CRN_TRY(h, crn::launch_gemm_mx8_rows<T>(a8, qs, wq, wsc, K, e, npad, st));
        return AEC_OK;
    }
    CRN_TRY(h, crn::launch_mx8_quant(a, bf.aq, bf.as, st));
    CRN_TRY(h, crn::launch_gemm_mx8<T>(bf.aq, bf.as, wq, wsc, K, e, npad, st));
    return AEC_OK;
}

// split-K workspace the MX conv GEMMs of a B-row step need (conv_ksplit per layer)
static void splitk_need(const aec_crn_handle* h, int64_t B, int64_t* bytes, int64_t* tiles) {
    const int* ch = h->cfg.conv_channels;
    *bytes = 0;
    *tiles = 0;
    auto need = [&](int64_t M, int N, int kpad) {
        *bytes = std::max(*bytes, crn::mx8_splitk_bytes(M, N, conv_ksplit(kpad)));
        *tiles = std::max(*tiles, crn::mx8_splitk_tiles(M, N));
    };
    for (int i = 0; i < h->L; ++i)
        if (h->enc[i].wq) need(B * (128 >> i), ch[i + 1], h->enc[i].kpad);
    for (int d = 0; d < h->L; ++d) {
        if (h->decf[d].wq) need(B * (256 >> (h->L - d)), h->decf[d].N, h->decf[d].kpad);
        for (int par = 0; par < 2; ++par) {
            const Packed& pk = h->dec[2 * d + par];
            if (pk.wq) need(B * (256 >> (h->L - d)), pk.N, pk.kpad);
        }
    }
}

// Batch forward: encoder levels 0-3 in one launch (crn_enc_batch_kernel) when the handle's
// levels have its shapes (bf16 storage, bf16 GEMMs on those levels); AEC_CRN_BATCH_ENC=0
// restores the four row GEMMs (A/B and the bit-equality test), =2 makes a handle whose levels do
// not fit fail with AEC_ERR_UNSUPPORTED (the test's proof that the fused path ran).  Returns the
// levels it ran.
template <typename T>
static int run_enc_batch_try(aec_crn_handle* h, const Bufs& bf, int64_t F, hipStream_t st, aec_status* s);
template <typename T>
static int run_enc_batch(aec_crn_handle* h, const Bufs& bf, int64_t F, hipStream_t st, aec_status* s) {
    *s = AEC_OK;
    const int mode = AEC_MODE_KNOB("AEC_CRN_BATCH_ENC", 1);
    if (mode == 0) return 0;
    const int n = run_enc_batch_try<T>(h, bf, F, st, s);
    if (n == 0 && *s == AEC_OK && mode == 2) {
        h->err = "AEC_CRN_BATCH_ENC=2: the encoder levels do not fit crn_enc_batch_kernel";
        *s = AEC_ERR_UNSUPPORTED;
    }
    return n;
}
template <typename T>
static int run_enc_batch_try(aec_crn_handle* h, const Bufs& bf, int64_t F, hipStream_t st, aec_status* s) {
    if (sizeof(T) != 2 || h->es != 2 || h->L < 5) return 0;
    const int* ch = h->cfg.conv_channels;
    crn::EncBatchArgs ea{};
    ea.x0 = reinterpret_cast<const bf16_t*>(bf.x0);
    ea.F = F;
    for (int i = 0; i < 4; ++i) {
        const Packed& pk = h->enc[i];
        if (pk.wq || pk.act != 1) return 0;
        crn::StreamEncLevel& L = ea.lev[i];
        L.w = reinterpret_cast<const bf16_t*>(pk.w);
        L.bias = pk.bias;
        L.alpha = pk.alpha;
        L.kpad = pk.kpad;
        L.N = pk.N;
        L.nchunk = (pk.K + 31) / 32;
        L.cin_shift = ilog2(i == 0 ? 8 : ch[i]);
        L.out = reinterpret_cast<bf16_t*>(bf.cat[i + 1]);
        L.ldo = 2 * ch[i + 1];
        L.choff = ch[i + 1];
        if (bf.cat8 && bf.cat8[i + 1] && pk.N % 128 == 0) {   // set_shadow's rule
            L.q8 = bf.cat8[i + 1];
            L.qs = bf.cats[i + 1];
        }
        if (pk.N != ch[i + 1]) return 0;
    }
    if (!crn::enc_batch_ok(ea)) return 0;
    const hipError_t e = crn::launch_enc_batch(ea, st);
    if (e != hipSuccess) {
        h->err = std::string("launch_enc_batch: ") + hipGetErrorString(e);
        *s = e == hipErrorOutOfMemory ? AEC_ERR_OOM : AEC_ERR_HIP;
        return 0;
    }
    return 4;
}

template <typename T>
static aec_status run_encoder(aec_crn_handle* h, const Bufs& bf, int64_t F, hipStream_t st, int first = 0,
                              bool batch = false) {
    using crn::RowEpi;
    using crn::RowSrc;
    aec_status s = AEC_OK;
    const int* ch = h->cfg.conv_channels;
    if (batch && first == 0) {
        first = run_enc_batch<T>(h, bf, F, st, &s);
        if (s != AEC_OK) return s;
    }
    for (int i = first; i < h->L; ++i) {
        const int Fin = 256 >> i, Fo = Fin / 2;
        const int cin = i == 0 ? 8 : ch[i];
        const int64_t ld_in = i == 0 ? 8 : 2 * ch[i];
        const int64_t choff = i == 0 ? 0 : ch[i];
        const Packed& pk = h->enc[i];
        RowSrc a{};
        a.src = i == 0 ? bf.x0 : bf.cat[i];
        a.M = F * Fo;
        a.K = pk.K;
        a.rshift = ilog2(Fo);
        a.rs_hi = Fin * ld_in;
        a.rs_lo = 2 * ld_in;
        a.kshift = ilog2(cin);
        a.ks = ld_in;
        a.pmul = 2;
        a.padd = -2;
        a.plim = Fin;
        a.base_off = choff - 2 * ld_in;
        a.src_elems = F * Fin * ld_in;
        const int64_t ldo = 2 * ch[i + 1];
        RowEpi e{bf.cat[i + 1], a.M, pk.N, a.rshift, Fo * ldo, ldo, ch[i + 1], pk.bias, pk.alpha, pk.act};
        set_shadow<T>(e, bf.cat8[i + 1], bf.cats[i + 1]);
        if (pk.wq) {                       // dtype 2: e4m3 rows + E8M0 scales, scaled-MFMA GEMM
            s = mx8_gemm<T>(h, a, i > 0 ? bf.cat8[i] : nullptr, i > 0 ? bf.cats[i] : nullptr, bf, pk.wq, pk.wsc,
                            pk.kpad, e, pk.npad8, st, true);
            if (s != AEC_OK) return s;
            continue;
        }
        CRN_TRY(h, (crn::launch_gemm_rows<T, T>(a, reinterpret_cast<const T*>(pk.w), pk.kpad,
                                                 (int)(pk.kpad * sizeof(T) / crn::kStageBytes), e, pk.npad, st)));
    }
    return AEC_OK;
}

// LSTM layer l input projection for F frames -> bf.gx [F][S][CELLS*4H]
template <typename T>
static aec_status run_lstm_input(aec_crn_handle* h, const Bufs& bf, int l, int64_t F, hipStream_t st) {
    using crn::RowEpi;
    using crn::RowSrc;
    const int* ch = h->cfg.conv_channels;
    const int L = h->L, H = h->H, S = h->S, C = h->CELLS, D = h->D, Q = h->Q;
    RowSrc a{};
    int64_t ld_in, choff;
    if (l == 0) {
        a.src = bf.cat[L];
        ld_in = 2 * ch[L];
        choff = ch[L];
    } else {
        a.src = bf.xn;
        ld_in = (int64_t)S * Q;
        choff = 0;
    }
    a.M = F * S;
    a.K = H;
    a.rshift = ilog2(S);
    a.rs_hi = D * ld_in;
    a.rs_lo = Q;
    a.kshift = ilog2(Q);
    a.ks = ld_in;
    a.pmul = 0;
    a.padd = 0;
    a.plim = D;
    a.base_off = choff;
    a.src_elems = F * D * ld_in;
    const Packed& ih = h->lih[l];
    RowEpi e{bf.gx, a.M, ih.N, 0, (int64_t)C * 4 * H, 0, 0, ih.bias, 0.f, 0};
    if (h->mx8)                            // e4m3 rows + E8M0 scales, scaled-MFMA GEMM
        return mx8_gemm<T>(h, a, l == 0 ? bf.cat8[L] : bf.xn8, l == 0 ? bf.cats[L] : bf.xns, bf, ih.wq, ih.wsc,
                           ih.kpad, e, ih.npad, st);
    CRN_TRY(h, (crn::launch_gemm_rows<T, T>(a, reinterpret_cast<const T*>(ih.w), ih.kpad,
                                             (int)(ih.kpad * sizeof(T) / crn::kStageBytes), e, ih.npad, st)));
    return AEC_OK;
}

// NavieComplexLSTM combination of layer l's h rows y [F][C][S][H] -> the next
// layer's input (xn) or the decoder's dec half of cat[L]
template <typename T>
static aec_status run_lstm_combine(aec_crn_handle* h, const Bufs& bf, int l, const void* y, int64_t F,
                                   hipStream_t st) {
    const int* ch = h->cfg.conv_channels;
    const int L = h->L, S = h->S, Q = h->Q;
    const bool last = l + 1 == h->nrnn;
    T* dst = reinterpret_cast<T*>(last ? bf.cat[L] : bf.xn);
    const int64_t ldd = last ? 2 * ch[L] : (int64_t)S * Q;
    uint8_t* q8 = sizeof(T) == 2 ? (last ? bf.cat8[L] : bf.xn8) : nullptr;
    uint8_t* qs = sizeof(T) == 2 ? (last ? bf.cats[L] : bf.xns) : nullptr;
    CRN_TRY(h, crn::launch_lstm_combine<T>(reinterpret_cast<const T*>(y), dst, F, h->H, h->CELLS, S, ilog2(Q),
                                           h->D * ldd, ldd, st, q8, qs));
    return AEC_OK;
}

template <typename T>
static aec_status run_decoder(aec_crn_handle* h, const Bufs& bf, int64_t F, hipStream_t st, int nd = -1, int d0 = 0) {
    using crn::RowEpi;
    using crn::RowSrc;
    const int* ch = h->cfg.conv_channels;
    const int L = h->L;
    for (int d = d0; d < (nd < 0 ? L : nd); ++d) {
        const int cl = L - d;
        const int Fin = 256 >> cl, Fo = 2 * Fin;
        const int64_t ld_in = 2 * ch[cl];
        if (h->decf[d].w) {                // both parities in one GEMM (pack_decoder_fused)
            const Packed& pk = h->decf[d];
            RowSrc a{};
            a.src = bf.cat[cl];
            a.M = F * Fin;
            a.K = pk.K;
            a.rshift = ilog2(Fin);
            a.rs_hi = Fin * ld_in;
            a.rs_lo = ld_in;
            a.kshift = ilog2(ld_in);
            a.ks = ld_in;
            a.pmul = 1;
            a.padd = -1;
            a.plim = Fin;
            a.base_off = -ld_in;
            a.src_elems = F * Fin * ld_in;
            if (cl == 1) {                 // the mask: row (f, i) -> bins 2i, 2i + 1 = 4 adjacent floats
                RowEpi e{bf.mask, a.M, pk.N, a.rshift, (int64_t)Fo * 2, 4, 0, pk.bias, pk.alpha, pk.act};
                CRN_TRY(h, (crn::launch_gemm_rows<T, float>(a, reinterpret_cast<const T*>(pk.w), pk.kpad,
                                                             (int)(pk.kpad * sizeof(T) / crn::kStageBytes), e,
                                                             pk.npad, st)));
                continue;
            }
            const int64_t ldo = 2 * ch[cl - 1];
            RowEpi e{bf.cat[cl - 1], a.M, pk.N, a.rshift, Fo * ldo, 2 * ldo, 0, pk.bias, pk.alpha, pk.act};
            e.nsplit = pk.N / 2;
            e.split_add = ldo;
            set_shadow<T>(e, bf.cat8[cl - 1], bf.cats[cl - 1]);
            if (pk.wq) {                   // dtype 2 (see conv_mx8)
                const aec_status s = mx8_gemm<T>(h, a, bf.cat8[cl], bf.cats[cl], bf, pk.wq, pk.wsc, pk.kpad, e,
                                                 pk.npad8, st, true);
                if (s != AEC_OK) return s;
                continue;
            }
            CRN_TRY(h, (crn::launch_gemm_rows<T, T>(a, reinterpret_cast<const T*>(pk.w), pk.kpad,
                                                     (int)(pk.kpad * sizeof(T) / crn::kStageBytes), e, pk.npad, st)));
            continue;
        }
        for (int par = 0; par < 2; ++par) {
            const Packed& pk = h->dec[2 * d + par];
            RowSrc a{};
            a.src = bf.cat[cl];
            a.M = F * Fin;
            a.K = pk.K;
            a.rshift = ilog2(Fin);
            a.rs_hi = Fin * ld_in;
            a.rs_lo = ld_in;
            a.kshift = ilog2(ld_in);
            a.ks = ld_in;
            a.pmul = 1;
            a.padd = par == 0 ? -1 : 0;
            a.plim = Fin;
            a.base_off = a.padd * ld_in;
            a.src_elems = F * Fin * ld_in;
            if (cl != 1) {
                const int64_t ldo = 2 * ch[cl - 1];
                RowEpi e{bf.cat[cl - 1], a.M, pk.N, a.rshift, Fo * ldo, 2 * ldo, par * ldo, pk.bias, pk.alpha, pk.act};
                set_shadow<T>(e, bf.cat8[cl - 1], bf.cats[cl - 1]);
                if (pk.wq) {               // dtype 2 (see conv_mx8)
                    const aec_status s = mx8_gemm<T>(h, a, bf.cat8[cl], bf.cats[cl], bf, pk.wq, pk.wsc, pk.kpad, e,
                                                     pk.npad8, st, true);
                    if (s != AEC_OK) return s;
                    continue;
                }
                CRN_TRY(h, (crn::launch_gemm_rows<T, T>(a, reinterpret_cast<const T*>(pk.w), pk.kpad,
                                                         (int)(pk.kpad * sizeof(T) / crn::kStageBytes), e, pk.npad,
                                                         st)));
            } else {
                RowEpi e{bf.mask, a.M, pk.N, a.rshift, (int64_t)Fo * 2, 4, (int64_t)par * 2, pk.bias, pk.alpha, pk.act};
                CRN_TRY(h, (crn::launch_gemm_rows<T, float>(a, reinterpret_cast<const T*>(pk.w), pk.kpad,
                                                             (int)(pk.kpad * sizeof(T) / crn::kStageBytes), e,
                                                             pk.npad, st)));
            }
        }
    }
    return AEC_OK;
}

static int mask_mode(const aec_crn_handle* h) {
    return h->cfg.version == 1 ? 1 : (h->cfg.masking_mode == 'E' ? 0 : h->cfg.masking_mode == 'C' ? 1 : 2);
}

// Device-wide order of persistent launches: a persistent grid needs every CU,
// so two of them co-resident (two handles / streams) could starve each other.
// Each launch waits for the previous one on this device.
static std::mutex g_persist_mu;
static hipEvent_t g_persist_ev[64] = {};

static aec_status run_persist(aec_crn_handle* h, int l, int32_t B, int64_t Tmax, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_persist_mu);
    hipEvent_t& ev = g_persist_ev[h->device & 63];
    if (!ev) CRN_TRY(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CRN_TRY(h, hipStreamWaitEvent(st, ev, 0));
    if (!h->persist_pending) {   // first persistent launch of this call: clear the error word
        CRN_TRY(h, hipMemsetAsync(h->psync + crn::kPersistErr, 0, sizeof(int), st));
        h->persist_pending = true;
    }
    // polls before a wave gives up; AEC_CRN_SPIN_LIMIT (read per call) forces a timeout in the tests
    const int spin = std::max(1, AEC_MODE_KNOB("AEC_CRN_SPIN_LIMIT", crn::kPersistSpinLimit));
    // AEC_CRN_PERSIST_STALL=1 (read per call, the timeout test's hook): the poll targets are never reached
    const int stall = AEC_MODE_KNOB("AEC_CRN_PERSIST_STALL", 0) != 0 ? (1 << 30) : 0;
    static const int pra = AEC_AB_KNOB("CRN_PERSIST_RA", 1);
    // one block per CU: 64 streams (two teams of 32 blocks) per 64 CUs, at most 256 streams per launch
    const int32_t chunk = 64 * std::min(4, h->num_cus / 64);
    for (int32_t b0 = 0; b0 < B; b0 += chunk) {
        const int nb = std::min<int32_t>(chunk, B - b0);
        crn::PersistArgs a{};
        a.whh = reinterpret_cast<const bf16_t*>(h->lhh[l].w);
        a.gx = reinterpret_cast<const bf16_t*>(h->gx);
        a.y = reinterpret_cast<bf16_t*>(h->y);
        a.sync = h->psync;
        a.B = B;
        a.b0 = b0;
        a.nb = nb;
        a.T = (int)Tmax;
        a.G = (nb + 63) / 64;
        a.spin_limit = spin;
        a.read_ahead = pra;
        a.stall = stall;
        // arrival counters only: the error word keeps any timeout of this call's earlier launches
        CRN_TRY(h, hipMemsetAsync(h->psync, 0, crn::kPersistCounters * sizeof(int), st));
        CRN_TRY(h, crn::launch_lstm_persist(a, st));
    }
    CRN_TRY(h, hipEventRecord(ev, st));
    return AEC_OK;
}

// After the last persistent launch of a call: copy the error word to the host
// (stream-ordered, right behind the LSTM stage) and record an event; before
// the call returns, the host waits for that event (persist_wait), so a
// timed-out grid fails the call that launched it.  The host then waits only
// until the LSTM stage has run: the decoder and back kernels are already
// queued behind it.
static aec_status persist_copy(aec_crn_handle* h, hipStream_t st) {
    if (!h->persist_pending) return AEC_OK;
    CRN_TRY(h, hipMemcpyAsync(h->perr_host, h->psync + crn::kPersistErr, sizeof(int), hipMemcpyDeviceToHost, st));
    CRN_TRY(h, hipEventRecord(h->perr_ev, st));
    return AEC_OK;
}

static aec_status persist_wait(aec_crn_handle* h) {
    if (!h->persist_pending) return AEC_OK;
    h->persist_pending = false;
    CRN_TRY(h, hipEventSynchronize(h->perr_ev));
    if (*h->perr_host) {
        // two timed-out calls in a row (co-residency lost, e.g. CUs held by another process): the
        // handle drops to the per-frame step kernel for every later call
        if (++h->persist_timeouts >= 2) h->persist = 0;
        return crn_fail(h, AEC_ERR_HIP,
                        "persistent LSTM recurrence: a block timed out waiting for its team (outputs invalid)");
    }
    h->persist_timeouts = 0;
    return AEC_OK;
}

// Batch forward, bf16 storage: decoder levels cl = 3, 2 in one launch (crn_dec_batch_kernel) when
// their shapes fit; AEC_CRN_BATCH_DEC=0 restores the two row GEMMs, =2 fails the call unless the
// fused kernel ran (the bit-equality test).  Returns true when it ran.
template <typename T>
static bool run_dec_batch(aec_crn_handle* h, const Bufs& bf, int64_t F, hipStream_t st, aec_status* s) {
    *s = AEC_OK;
    const int mode = AEC_MODE_KNOB("AEC_CRN_BATCH_DEC", 1);
    if (mode == 0) return false;
    bool ok = sizeof(T) == 2 && h->es == 2 && h->L >= 4;
    crn::DecBatchArgs da{};
    if (ok) {
        const int* ch = h->cfg.conv_channels;
        da.F = F;
        for (int l = 0; l < 2; ++l) {
            const int cl = 3 - l, d = h->L - cl;
            const Packed& pk = h->decf[d];
            crn::StreamDecLevel& L = da.lev[l];
            if (!pk.w || pk.wq || pk.N != 2 * ch[cl - 1]) ok = false;
            L.w = reinterpret_cast<const bf16_t*>(pk.w);
            L.bias = pk.bias;
            L.alpha = pk.alpha;
            L.act = pk.act;
            L.kpad = pk.kpad;
            L.N = pk.N;
            L.nchunk = (pk.K + 31) / 32;
            L.cin_shift = ilog2(2 * ch[cl]);
            L.src = reinterpret_cast<const bf16_t*>(bf.cat[cl]);
        }
        da.out = reinterpret_cast<bf16_t*>(bf.cat[1]);
        da.ldo1 = 2 * ch[1];
        ok = ok && crn::dec_batch_ok(da);
    }
    if (!ok) {
        if (mode == 2) {
            h->err = "AEC_CRN_BATCH_DEC=2: decoder levels 3, 2 do not fit crn_dec_batch_kernel";
            *s = AEC_ERR_UNSUPPORTED;
        }
        return false;
    }
    const hipError_t e = crn::launch_dec_batch(da, st);
    if (e != hipSuccess) {
        h->err = std::string("launch_dec_batch: ") + hipGetErrorString(e);
        *s = e == hipErrorOutOfMemory ? AEC_ERR_OOM : AEC_ERR_HIP;
        return false;
    }
    return true;
}

template <typename T>
static aec_status run(aec_crn_handle* h, const float* mic, const float* far, int32_t B, int64_t ld, int64_t Tmax,
                      float* out, int64_t ld_out, float* spec, float* mask_out, hipStream_t st) {
    const int64_t BT = (int64_t)B * Tmax;
    const Bufs bf{h->x0, h->cat.data(), h->gx, h->xn, h->mask, h->aq, h->as, h->cat8.data(), h->cats.data(), h->xn8,
                  h->xns};
    const int H = h->H, S = h->S, C = h->CELLS;
    const bool persist = sizeof(T) == 2 && h->persist && h->psync && crn::persist_supported(H, C, S, h->num_cus);
    mark(h, st);
    // front: X0 [Tmax][B][256][8]
    const aec_crn_config& c = h->cfg;
    crn::FrontArgs fa{mic, far, ld, h->d_len, Tmax, h->d_tab, h->x0, nullptr};
    if (c.nlms_taps > 0) fa.rows = h->nrows;
    CRN_TRY(h, crn::launch_front<T>(fa, B, st));
    if (c.nlms_taps > 0) {   // FD-NLMS: rows -> E rows (one block per stream) -> X0
        CRN_TRY(h, aec::launch_nlms_recursion(h->nrows, h->espec, h->d_len, Tmax, c.nlms_taps, c.nlms_mu, c.nlms_beta,
                                              c.nlms_delta, 0, B, h->ndummy, st));
        crn::RowsX0Args xa{h->nrows, h->espec, h->d_len, Tmax, h->x0, B};
        CRN_TRY(h, crn::launch_rows_x0<T>(xa, st));
    }
    mark(h, st);
    aec_status s = run_encoder<T>(h, bf, BT, st, 0, true);
    if (s != AEC_OK) return s;
    mark(h, st);
    for (int l = 0; l < h->nrnn; ++l) {
        s = run_lstm_input<T>(h, bf, l, BT, st);
        if (s != AEC_OK) return s;
        const int64_t ystride = (int64_t)B * C * S * H, gstride = (int64_t)B * S * C * 4 * H;   // per frame
        if (persist) {   // all Tmax frames of the layer in one launch per 256 streams
            s = run_persist(h, l, B, Tmax, st);
            if (s != AEC_OK) return s;
            s = run_lstm_combine<T>(h, bf, l, h->y, BT, st);
            if (s != AEC_OK) return s;
            continue;
        }
        for (int64_t t = 0; t < Tmax; ++t) {
            crn::StepArgs sa{h->lhh[l].w, reinterpret_cast<const T*>(h->gx) + t * gstride,
                             reinterpret_cast<const T*>(h->y) + (t > 0 ? t - 1 : 0) * ystride,
                             reinterpret_cast<T*>(h->y) + t * ystride, h->cst, B, H, t == 0, 0};
            CRN_TRY(h, crn::launch_lstm_step<T>(sa, C, S, st));
        }
        s = run_lstm_combine<T>(h, bf, l, h->y, BT, st);
        if (s != AEC_OK) return s;
    }
    s = persist_copy(h, st);
    if (s != AEC_OK) return s;
    mark(h, st);
    // bf16: the mask level runs inside the back kernel (no f32 mask round trip) unless the
    // caller wants the mask itself (AEC_CRN_BACK_MASK=0: the row GEMM, A/B and bit-equality)
    const Packed& pm = h->decf[h->L - 1];
    const bool mask_in_back = sizeof(T) == 2 && AEC_MODE_KNOB("AEC_CRN_BACK_MASK", 1) != 0 && pm.w && !mask_out &&
                              (out || spec) && pm.N == 4 && pm.kpad <= 128 && pm.kpad % 32 == 0 && pm.act != 1;
    {
        // decoder levels cl = L .. 4 as row GEMMs, cl = 3, 2 fused when they fit, then the mask
        // level (cl = 1) as a GEMM unless the back kernel computes it
        const int Ld = h->L, d3 = std::max(0, Ld - 3);
        s = run_decoder<T>(h, bf, BT, st, d3);
        if (s != AEC_OK) return s;
        const bool fused = run_dec_batch<T>(h, bf, BT, st, &s);
        if (s != AEC_OK) return s;
        s = run_decoder<T>(h, bf, BT, st, mask_in_back ? Ld - 1 : Ld, fused ? Ld - 1 : d3);
        if (s != AEC_OK) return s;
    }
    mark(h, st);
    if (out || spec) {
        crn::BackArgs ba{mic, ld, h->d_len, Tmax, h->d_tab, reinterpret_cast<const float2*>(h->mask), out, ld_out,
                         reinterpret_cast<float2*>(spec)};
        if (c.nlms_taps > 0) ba.espec = h->espec;
        if (mask_in_back) {
            ba.dm_in = reinterpret_cast<const bf16_t*>(h->cat[1]);
            ba.dm_w = reinterpret_cast<const bf16_t*>(pm.w);
            ba.dm_bias = pm.bias;
            ba.dm_kpad = pm.kpad;
            ba.dm_cin_shift = ilog2(2 * h->cfg.conv_channels[1]);
            ba.dm_act = pm.act;
        }
        CRN_TRY(h, crn::launch_back(ba, B, mask_mode(h), st));
    }
    if (mask_out)   // internal frames are t-major ([Tmax][B]); the ABI's mask is [B][Tmax]
        for (int b = 0; b < B; ++b)
            CRN_TRY(h, hipMemcpy2DAsync(mask_out + (size_t)b * Tmax * 512, 512 * sizeof(float), h->mask + (size_t)b * 512,
                                        (size_t)B * 512 * sizeof(float), 512 * sizeof(float), (size_t)Tmax,
                                        hipMemcpyDeviceToDevice, st));
    mark(h, st);
    return AEC_OK;
}

// --------------------------------------------------------------------------
// streaming: one 256-sample hop per stream per call (aec_crn_stream_*)
// --------------------------------------------------------------------------
struct StreamState {
    int32_t B = 0;
    int64_t k = 0;                       // hops consumed since open / reset-all
    // per-hop launch mode of this handle's streams: 0 direct launches, 1 hipGraph replay
    // (AEC_CRN_GRAPH read at stream_open, aec_crn_stream_set_graph afterwards); hops run each way
    int graph_mode = 0;
    int64_t graph_replays = 0, direct_hops = 0;
    std::vector<void*> allocs;
    void* x0 = nullptr;
    std::vector<void*> cat;
    void* gx = nullptr;
    void* xn = nullptr;
    float* mask = nullptr;
    uint8_t* aq = nullptr;               // dtype 2 (see Bufs)
    uint8_t* as = nullptr;
    std::vector<uint8_t*> cat8, cats;
    uint8_t* xn8 = nullptr;
    uint8_t* xns = nullptr;
    void* xnb = nullptr;                 // MX layer step, rnn_layers >= 3: the second xn set (bf16 rows,
    uint8_t* xn8b = nullptr;             //   e4m3 shadow, scales) the odd middle layers write
    uint8_t* xnsb = nullptr;
    float* skp = nullptr;                // split-K partial tiles / tile counters of the MX conv GEMMs (Bufs)
    int* skc = nullptr;
    int64_t sk_bytes = 0;
    int32_t skc_n = 0;
    void* ring_y[8][2] = {};             // per LSTM layer: h ring (two frames)
    uint8_t* ring_q[8][2] = {};          // dtype 2 MX layer step: h ring as e4m3 [B][C][S][H] + E8M0 [B][C][S][H/32]
    uint8_t* ring_s[8][2] = {};
    float* hx = nullptr;                 //   h_t f32 [B][C][S][H] (cell-pair hand-off)
    int* mx_cnt = nullptr;               //   arrival counters (zero between launches)
    bool mx_step = false;
    float* cst[8] = {};                  // per LSTM layer: c
    float* hop = nullptr;                // [2 parity][2 signal][B][256] hop ring (mic, far): the front kernel
                                         //   copies each call's hops in, for the next call and the back kernel
    float* tail = nullptr;               // [B][256] overlap-add tail
    float2* nrows = nullptr;             // NLMS: packed rows [B][2][256]
    float2* nstate = nullptr;            //       recursion state [B][2*taps][256]
    float2* espec = nullptr;             //       E rows [B][256]
    // one hipGraph per ring parity; the caller's hop / output buffers change per call, so the
    // front and back kernel nodes get this call's pointers by hipGraphExecKernelNodeSetParams
    // (a host-side update: no copy kernels in the step)
    hipGraph_t gsrc[2] = {nullptr, nullptr};
    hipGraphExec_t graph[2] = {nullptr, nullptr};
    hipGraphNode_t front_node[2] = {nullptr, nullptr}, back_node[2] = {nullptr, nullptr};
    crn::StreamFrontArgs front_args[2];
    crn::StreamBackArgs back_args[2];
    // bf16 / fp8: the front, the NLMS step and the narrow encoder levels 0 .. enc_nlev-1 as one
    // launch (crn_stream_enc_kernel); its graph node is front_node (AEC_CRN_STREAM_FUSE=0: off)
    int enc_nlev = 0;
    crn::StreamEncArgs enc_args[2];
    // bf16 / fp8: the last three decoder levels, the mask, irFFT and overlap-add as one launch
    // (crn_stream_dec_kernel); its graph node is back_node (AEC_CRN_STREAM_FUSE=0: off)
    bool dec_fused = false;
    bool dec_mx = false;                 // + decoder cl = 4 (MX-fp8) inside it (AEC_CRN_STREAM_FUSE bit 3)
    bool enc_mx = false;                 // + encoder level 4 (MX-fp8) inside the fused front (bit 4)
    crn::StreamDecArgs dec_args[2];
    hipStream_t cap = nullptr;           // capture stream
};

// the caller's buffers of one aec_crn_stream_step call
struct StreamIo {
    const float* mic;
    const float* far;
    int64_t ld_in;
    float* out;
    int64_t ld_out;
};

static void stream_free(aec_crn_handle* h) {
    if (!h->ss) return;
    for (int p = 0; p < 2; ++p) {
        if (h->ss->graph[p]) (void)hipGraphExecDestroy(h->ss->graph[p]);
        if (h->ss->gsrc[p]) (void)hipGraphDestroy(h->ss->gsrc[p]);
    }
    for (void* p : h->ss->allocs) (void)hipFree(p);
    if (h->ss->cap) (void)hipStreamDestroy(h->ss->cap);
    delete h->ss;
    h->ss = nullptr;
}

// the kernel node the last launch on a capturing stream added (null when not capturing)
static hipGraphNode_t last_node(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    if (hipStreamGetCaptureInfo_v2(st, &cs, nullptr, nullptr, &deps, &nd) != hipSuccess) return nullptr;
    return cs == hipStreamCaptureStatusActive && nd == 1 ? deps[0] : nullptr;
}

// dtype 2, NavieComplexLSTM, per-hop: layer l as ONE launch (lstm_step_mx8_kernel): [x | h]
// against [W_ih | W_hh] on the scaled MFMA, the cell update and the combination.  x is read
// in place from its MX-fp8 shadow (the encoder's / previous combination's epilogue), or,
// without one (AEC_CRN_MX8_SHADOW=0), quantised first into bf.aq / bf.as by the same rule
// (*quant: that pass's rows).  A middle layer (neither first nor last, rnn_layers >= 3) reads
// its input from one xn set and writes the other: blocks that finish early would otherwise
// overwrite rows other blocks of the same launch still load.
static void mx_step_args(aec_crn_handle* h, const StreamState& ss, const Bufs& bf, int l, int par,
                         crn::StepMxArgs& ma, crn::RowSrc* quant) {
    const int* ch = h->cfg.conv_channels;
    const int L = h->L, H = h->H, S = h->S, D = h->D, Q = h->Q, B = ss.B;
    const bool last = l + 1 == h->nrnn;
    const bool in_b = l > 0 && ((l - 1) & 1), out_b = (l & 1) != 0;
    void* xn_in = in_b ? ss.xnb : bf.xn;
    void* xn_out = out_b ? ss.xnb : bf.xn;
    uint8_t* xn8_in = in_b ? ss.xn8b : bf.xn8;
    uint8_t* xns_in = in_b ? ss.xnsb : bf.xns;
    ma = crn::StepMxArgs{};
    ma.wq = h->lcat[l].wq;
    ma.wsc = h->lcat[l].wsc;
    ma.bias = h->lih[l].bias;
    // x rows (b, s): the bf16 GEMM's implicit LSTM-input rows (run_lstm_input)
    const int64_t ld_in = l == 0 ? 2 * ch[L] : (int64_t)S * Q;
    const int64_t choff = l == 0 ? ch[L] : 0;
    const uint8_t* x8 = l == 0 ? bf.cat8[L] : xn8_in;
    const uint8_t* xs = l == 0 ? bf.cats[L] : xns_in;
    if (quant) *quant = crn::RowSrc{};
    if (x8) {
        ma.xq = x8;
        ma.xs = xs;
        ma.x_f = D * ld_in;
        ma.x_s = Q;
        ma.x_t = ld_in;
        ma.x_sh = ilog2(Q);
        ma.x_0 = choff;
        ma.x_elems = (int64_t)B * D * ld_in;
    } else {
        if (quant) {
            crn::RowSrc& a = *quant;
            a.src = l == 0 ? bf.cat[L] : xn_in;
            a.M = (int64_t)B * S;
            a.K = H;
            a.rshift = ilog2(S);
            a.rs_hi = D * ld_in;
            a.rs_lo = Q;
            a.kshift = ilog2(Q);
            a.ks = ld_in;
            a.plim = D;
            a.base_off = choff;
            a.src_elems = (int64_t)B * D * ld_in;
        }
        ma.xq = bf.aq;                              // dense rows [(b, s)][H]
        ma.xs = bf.as;
        ma.x_f = (int64_t)S * H;
        ma.x_s = H;
        ma.x_t = 0;
        ma.x_sh = ilog2(H);
        ma.x_0 = 0;
        ma.x_elems = (int64_t)B * S * H;
    }
    ma.hq_prev = ss.ring_q[l][1 - par];
    ma.hs_prev = ss.ring_s[l][1 - par];
    ma.hq_cur = ss.ring_q[l][par];
    ma.hs_cur = ss.ring_s[l][par];
    ma.cst = ss.cst[l];
    ma.hx = ss.hx;
    ma.cnt = ss.mx_cnt;
    ma.dst = reinterpret_cast<crn::bf16_t*>(last ? bf.cat[L] : xn_out);
    ma.ldd = last ? 2 * ch[L] : (int64_t)S * Q;
    ma.ldf = D * ma.ldd;
    ma.dshift = ilog2(Q);
    ma.q8 = last ? bf.cat8[L] : out_b ? ss.xn8b : bf.xn8;
    ma.qs = last ? bf.cats[L] : out_b ? ss.xnsb : bf.xns;
    ma.B = B;
    ma.H = H;
}

static aec_status run_lstm_mx_step(aec_crn_handle* h, StreamState& ss, const Bufs& bf, int l, int par, hipStream_t st) {
    crn::StepMxArgs ma;
    crn::RowSrc q;
    mx_step_args(h, ss, bf, l, par, ma, &q);
    if (q.src) CRN_TRY(h, crn::launch_mx8_quant(q, bf.aq, bf.as, st));
    CRN_TRY(h, crn::launch_lstm_step_mx8(ma, st));
    return AEC_OK;
}

// the fused front's level table (stream_open checked the shapes: stream_enc_levels)
static crn::StreamEncArgs stream_enc_args(aec_crn_handle* h, int B) {
    StreamState& ss = *h->ss;
    const int* ch = h->cfg.conv_channels;
    crn::StreamEncArgs ea{};
    ea.tab = h->d_tab;
    ea.B = B;
    if (h->cfg.nlms_taps > 0) {
        ea.state = ss.nstate;
        ea.espec = ss.espec;
        ea.mu = h->cfg.nlms_mu;
        ea.beta = h->cfg.nlms_beta;
        ea.delta = h->cfg.nlms_delta;
    }
    ea.nlev = ss.enc_nlev;
    if (ss.enc_mx) {
        const Packed& pk = h->enc[4];
        ea.mx4.wq = pk.wq;
        ea.mx4.wsc = pk.wsc;
        ea.mx4.bias = pk.bias;
        ea.mx4.alpha = pk.alpha;
        ea.mx4.out = reinterpret_cast<bf16_t*>(ss.cat[5]);
        ea.mx4.ldo = 2 * ch[5];
        ea.mx4.choff = ch[5];
        ea.mx4.q8 = ss.cat8[5];
        ea.mx4.qs = ss.cats[5];
    }
    for (int i = 0; i < ss.enc_nlev; ++i) {
        const Packed& pk = h->enc[i];
        crn::StreamEncLevel& L = ea.lev[i];
        L.w = reinterpret_cast<const bf16_t*>(pk.w);
        L.bias = pk.bias;
        L.alpha = pk.alpha;
        L.kpad = pk.kpad;
        L.N = pk.N;
        L.nchunk = (pk.K + 31) / 32;
        L.cin_shift = ilog2(i == 0 ? 8 : ch[i]);
        L.out = reinterpret_cast<bf16_t*>(ss.cat[i + 1]);
        L.ldo = 2 * ch[i + 1];
        L.choff = ch[i + 1];
        if (shadow_level(h, i + 1)) {
            L.q8 = ss.cat8[i + 1];
            L.qs = ss.cats[i + 1];
        }
    }
    return ea;
}

// the fused back's level table: decoder levels cl = 3, 2, 1 (decf[L - 3 .. L - 1])
static crn::StreamDecArgs stream_dec_args(aec_crn_handle* h, int B) {
    StreamState& ss = *h->ss;
    const int* ch = h->cfg.conv_channels;
    crn::StreamDecArgs da{};
    for (int l = 0; l < 3; ++l) {
        const int cl = 3 - l, d = h->L - cl;
        const Packed& pk = h->decf[d];
        crn::StreamDecLevel& L = da.lev[l];
        L.w = reinterpret_cast<const bf16_t*>(pk.w);
        L.bias = pk.bias;
        L.alpha = pk.alpha;
        L.act = pk.act;
        L.kpad = pk.kpad;
        L.N = pk.N;
        L.nchunk = (pk.K + 31) / 32;
        L.cin_shift = ilog2(2 * ch[cl]);
        L.src = reinterpret_cast<const bf16_t*>(ss.cat[cl]);
    }
    da.tab = h->d_tab;
    da.espec = h->cfg.nlms_taps > 0 ? ss.espec : nullptr;
    da.tail = ss.tail;
    da.B = B;
    return da;
}

// the last three decoder levels crn_stream_dec_kernel can take (fused-parity bf16 GEMMs, the
// map shapes of configs.net_conf's narrow levels)
static bool stream_dec_ok(const aec_crn_handle* h) {
    if (h->es != 2 || h->L < 3) return false;
    // AEC_CRN_STREAM_FUSE (A/B knob; unset = every bit on, i.e. 31): bit 0 fused front (encoder
    // levels 0-2), bit 1 fused back (decoder cl = 3..1 + mask + irFFT), bit 2 encoder level 3 in the
    // front, bit 3 decoder cl = 4 (MX) in the back, bit 4 encoder level 4 (MX) in the front; the MX
    // folds (bits 3, 4) are further limited to streams <= CUs at stream_open
    if (!(AEC_MODE_KNOB("AEC_CRN_STREAM_FUSE", 31) & 2)) return false;
    const int* ch = h->cfg.conv_channels;
    const int caps[3] = {crn::kStreamDecChunks0, crn::kStreamDecChunks1, crn::kStreamDecChunks2};
    for (int l = 0; l < 3; ++l) {
        const int cl = 3 - l, d = h->L - cl, Fin = 256 >> cl;
        const Packed& pk = h->decf[d];
        const int NT = (pk.N + 15) / 16;
        if (!pk.w || pk.wq || (pk.K + 31) / 32 != caps[l] || pk.kpad < 32 * ((pk.K + 31) / 32) || (Fin / 16) * NT != 8 ||
            4 % NT || Fin * 2 * ch[cl] > 4096 || ilog2(2 * ch[cl]) != 7 - l)
            return false;
        if (l < 2 && (pk.act != 1 || pk.N != 2 * ch[cl - 1] || pk.N % 32)) return false;
        if (l == 2 && (pk.N != 4 || pk.act == 1)) return false;
    }
    return true;
}

// decoder cl = 4 inside the fused back (MX-fp8 step, AEC_CRN_STREAM_FUSE bit 3, default on): its
// fused-parity MX GEMM at net_conf's shape (16 input bins x 256 channels -> 2 x 64 columns, K = 768)
// reading cat[4]'s shadow, split into 1 or 2 K slices
static bool stream_dec_mx_ok(const aec_crn_handle* h) {
    if (!(AEC_MODE_KNOB("AEC_CRN_STREAM_FUSE", 31) & 8)) return false;
    if (h->L < 5 || !h->ss) return false;
    const int* ch = h->cfg.conv_channels;
    const Packed& pk = h->decf[h->L - 4];
    const int ks = conv_ksplit(pk.kpad);
    return pk.wq && pk.wsc && pk.act == 1 && pk.N == 128 && pk.K == 768 && pk.kpad == 768 && ch[4] == 128 &&
           ch[3] == 64 && shadow_level(h, 4) && h->ss->cat8.size() > 4 && h->ss->cat8[4] && h->ss->cats[4] && (ks == 1 || ks == 2);
}

// encoder level 4 inside the fused front (MX-fp8 step, AEC_CRN_STREAM_FUSE bit 4, default on): its
// MX GEMM at net_conf's shape (8 output bins x 256 channels, K = 5 taps x 128, one K slice) on level
// 3's shadow, its output with a shadow for level 5
static bool stream_enc_mx_ok(const aec_crn_handle* h) {
    if (!(AEC_MODE_KNOB("AEC_CRN_STREAM_FUSE", 31) & 16)) return false;
    if (h->L < 6 || !h->ss) return false;
    const int* ch = h->cfg.conv_channels;
    const Packed& pk = h->enc[4];
    const StreamState& ss = *h->ss;
    return pk.wq && pk.wsc && pk.act == 1 && pk.N == 256 && pk.K == 640 && pk.kpad == 640 && ch[4] == 128 &&
           ch[5] == 256 && conv_ksplit(pk.kpad) == 1 && ss.cat8.size() > 5 && ss.cat8[4] && ss.cats[4] &&
           ss.cat8[5] && ss.cats[5];
}

// leading encoder levels crn_stream_enc_kernel can take: bf16 GEMM (not MX), PReLU, 8 output tiles
// of 16 bins x 16 channels, K <= 160, no MX shadow on the output
static int stream_enc_levels(const aec_crn_handle* h) {
    if (h->es != 2) return 0;
    const int fuse = AEC_MODE_KNOB("AEC_CRN_STREAM_FUSE", 31);
    if (!(fuse & 1)) return 0;
    const int* ch = h->cfg.conv_channels;
    int n = 0;
    // levels 0-2 together, at net_conf's shapes (crn_stream_enc_kernel's compile-time chunk counts)
    const int nc[3] = {2, 3, 5};
    for (int i = 0; i < std::min(3, h->L); ++i) {
        const Packed& pk = h->enc[i];
        const int cin = i == 0 ? 8 : ch[i];
        if (pk.wq || pk.act != 1 || pk.N != (16 << i) || cin != (8 << i) || (pk.K + 31) / 32 != nc[i] ||
            pk.kpad < 32 * nc[i] || shadow_level(h, i + 1))
            return 0;
        ++n;
    }
    if (n < 3) return 0;
    // level 3 (16 x 128 from the 32 x 64 map; its MX shadow written in the kernel): AEC_CRN_STREAM_FUSE bit 2
    if (n == 3 && h->L > 4 && (fuse & 4)) {
        const Packed& pk = h->enc[3];
        const int nc = (pk.K + 31) / 32;
        if (!pk.wq && pk.act == 1 && pk.N == 128 && ch[3] == 64 && ch[4] == 128 && nc == crn::kStreamEncChunks3 &&
            pk.kpad >= 32 * nc)
            ++n;
    }
    return n;
}

template <typename T>
static aec_status stream_launches(aec_crn_handle* h, int par, const StreamIo& io, hipStream_t st) {
    StreamState& ss = *h->ss;
    const int B = ss.B;
    const Bufs bf{ss.x0,       ss.cat.data(), ss.gx,   ss.xn,  ss.mask,     ss.aq,    ss.as, ss.cat8.data(),
                  ss.cats.data(), ss.xn8,      ss.xns, ss.skp, ss.skc, ss.sk_bytes, ss.skc_n};
    float* cur_mic = ss.hop + (size_t)(par * 2 + 0) * B * 256;
    float* cur_far = ss.hop + (size_t)(par * 2 + 1) * B * 256;
    const float* prev_mic = ss.hop + (size_t)((1 - par) * 2 + 0) * B * 256;
    const float* prev_far = ss.hop + (size_t)((1 - par) * 2 + 1) * B * 256;
    const aec_crn_config& c = h->cfg;
    // the frame = [previous hop (ring), this call's hop (caller's buffer)]; the front kernel
    // copies this hop into the ring slot of this parity
    int first = 0;
    if (ss.enc_nlev > 0) {
        crn::StreamEncArgs ea = stream_enc_args(h, B);
        ea.prev_mic = prev_mic;
        ea.cur_mic = io.mic;
        ea.prev_far = prev_far;
        ea.cur_far = io.far;
        ea.ld_cur = io.ld_in;
        ea.save_mic = cur_mic;
        ea.save_far = cur_far;
        CRN_TRY(h, crn::launch_stream_enc(ea, c.nlms_taps, st));
        ss.front_node[par] = last_node(st);
        ss.enc_args[par] = ea;
        // AEC_CRN_ENC_MX_RERUN=1 (debugging only): the level-4 GEMM runs after the fused front anyway
        static const bool rerun = AEC_AB_KNOB("AEC_CRN_ENC_MX_RERUN", 0) != 0;
        first = ss.enc_nlev + (ss.enc_mx && !rerun ? 1 : 0);
    } else {
        crn::StreamFrontArgs fa{prev_mic, io.mic, prev_far, io.far, h->d_tab, ss.x0, B};
        fa.ld_cur = io.ld_in;
        fa.save_mic = cur_mic;
        fa.save_far = cur_far;
        if (c.nlms_taps > 0) fa.rows = ss.nrows;
        CRN_TRY(h, crn::launch_stream_front<T>(fa, st));
        ss.front_node[par] = last_node(st);
        ss.front_args[par] = fa;
        if (c.nlms_taps > 0) {
            crn::StreamNlmsArgs na{ss.nrows, ss.nstate, ss.espec, ss.x0, B, c.nlms_mu, c.nlms_beta, c.nlms_delta};
            CRN_TRY(h, crn::launch_stream_nlms<T>(na, c.nlms_taps, st));
        }
    }
    aec_status s = run_encoder<T>(h, bf, B, st, first);
    if (s != AEC_OK) return s;
    for (int l = 0; l < h->nrnn; ++l) {
        if (ss.mx_step) {
            if constexpr (sizeof(T) == 2) {
                s = run_lstm_mx_step(h, ss, bf, l, par, st);
                if (s != AEC_OK) return s;
            }
            continue;
        }
        s = run_lstm_input<T>(h, bf, l, B, st);
        if (s != AEC_OK) return s;
        crn::StepArgs sa{h->lhh[l].w, ss.gx, ss.ring_y[l][1 - par], ss.ring_y[l][par], ss.cst[l], B, h->H, 0, 0};
        CRN_TRY(h, crn::launch_lstm_step<T>(sa, h->CELLS, h->S, st));
        s = run_lstm_combine<T>(h, bf, l, ss.ring_y[l][par], B, st);
        if (s != AEC_OK) return s;
    }
    if (ss.dec_fused) {
        s = run_decoder<T>(h, bf, B, st, h->L - (ss.dec_mx ? 4 : 3));
        if (s != AEC_OK) return s;
        crn::StreamDecArgs da = stream_dec_args(h, B);
        if (ss.dec_mx) {
            const Packed& pk = h->decf[h->L - 4];
            da.mx = crn::StreamDecMxLevel{pk.wq, pk.wsc, pk.bias, pk.alpha, ss.cat8[4], ss.cats[4], conv_ksplit(pk.kpad)};
        }
        da.prev_mic = prev_mic;
        da.cur_mic = cur_mic;
        da.out = io.out;
        da.ld_out = io.ld_out;
        CRN_TRY(h, crn::launch_stream_dec(da, mask_mode(h), st));
        ss.back_node[par] = last_node(st);
        ss.dec_args[par] = da;
        return AEC_OK;
    }
    s = run_decoder<T>(h, bf, B, st);
    if (s != AEC_OK) return s;
    crn::StreamBackArgs ba{prev_mic, cur_mic, h->d_tab, reinterpret_cast<const float2*>(ss.mask), ss.tail, io.out, B};
    ba.ld_out = io.ld_out;
    if (c.nlms_taps > 0) ba.espec = ss.espec;
    CRN_TRY(h, crn::launch_stream_back(ba, mask_mode(h), st));
    ss.back_node[par] = last_node(st);
    ss.back_args[par] = ba;
    return AEC_OK;
}

// point the captured front / back kernel nodes of parity `par` at this call's buffers
static aec_status stream_set_io(aec_crn_handle* h, int par, const StreamIo& io) {
    StreamState& ss = *h->ss;
    crn::StreamFrontArgs& fa = ss.front_args[par];
    crn::StreamEncArgs& ea = ss.enc_args[par];
    crn::StreamBackArgs& ba = ss.back_args[par];
    crn::StreamDecArgs& da = ss.dec_args[par];
    const bool fused = ss.enc_nlev > 0;
    const float* cm = fused ? ea.cur_mic : fa.cur_mic;
    const float* cf = fused ? ea.cur_far : fa.cur_far;
    const int64_t cl = fused ? ea.ld_cur : fa.ld_cur;
    const float* co = ss.dec_fused ? da.out : ba.out;
    const int64_t clo = ss.dec_fused ? da.ld_out : ba.ld_out;
    if (cm == io.mic && cf == io.far && cl == io.ld_in && co == io.out && clo == io.ld_out) return AEC_OK;
    fa.cur_mic = ea.cur_mic = io.mic;
    fa.cur_far = ea.cur_far = io.far;
    fa.ld_cur = ea.ld_cur = io.ld_in;
    ba.out = da.out = io.out;
    ba.ld_out = da.ld_out = io.ld_out;
    hipKernelNodeParams kp{};
    CRN_TRY(h, hipGraphKernelNodeGetParams(ss.front_node[par], &kp));
    void* fargs[] = {fused ? static_cast<void*>(&ea) : static_cast<void*>(&fa)};
    kp.kernelParams = fargs;
    kp.extra = nullptr;
    CRN_TRY(h, hipGraphExecKernelNodeSetParams(ss.graph[par], ss.front_node[par], &kp));
    CRN_TRY(h, hipGraphKernelNodeGetParams(ss.back_node[par], &kp));
    void* bargs[] = {ss.dec_fused ? static_cast<void*>(&da) : static_cast<void*>(&ba)};
    kp.kernelParams = bargs;
    kp.extra = nullptr;
    CRN_TRY(h, hipGraphExecKernelNodeSetParams(ss.graph[par], ss.back_node[par], &kp));
    return AEC_OK;
}
extern "C" {

size_t aec_crn_param_count(const aec_crn_config* cfg) { return cfg ? param_count(*cfg) : 0; }

const char* aec_crn_last_error(const aec_crn_handle* h) { return h ? h->err.c_str() : "null handle"; }

aec_status aec_crn_create(const aec_crn_config* cfg, const float* params, size_t n, int32_t device,
                          aec_crn_handle** out) {
    if (!cfg || !out) return AEC_ERR_INVALID_ARG;
    *out = nullptr;
    const std::string why = check_cfg(*cfg);
    if (!why.empty()) return AEC_ERR_UNSUPPORTED;
    aec_crn_handle* h = new (std::nothrow) aec_crn_handle();
    if (!h) return AEC_ERR_OOM;
    h->cfg = *cfg;
    h->device = device;
    h->L = cfg->n_layers;
    h->D = 256 >> h->L;
    h->es = cfg->dtype == 0 ? 4 : 2;
    h->mx8 = cfg->dtype == 2;
    if (cfg->version == 1) {
        h->H = cfg->conv_channels[h->L] * 4;
        h->S = h->CELLS = 1;
        h->nrnn = 1;
    } else {
        h->H = cfg->hidden_dim * cfg->conv_channels[h->L] / 2;
        h->S = h->CELLS = 2;
        h->nrnn = cfg->rnn_layers;
    }
    h->Q = h->H / h->D;
    if (h->mx8 && (h->H % 128 || h->Q % 32)) {     // MX blocks of 32 k inside one tap, 128-k stages
        delete h;
        return AEC_ERR_UNSUPPORTED;
    }
    auto bail = [&](aec_status s) {
        aec_crn_destroy(h);
        return s;
    };
    if (h->H % 32 || ilog2(h->Q) < 0) return bail(AEC_ERR_UNSUPPORTED);
    aec::DeviceGuard dg(device);
    if (dg.err != hipSuccess) return bail(AEC_ERR_HIP);
    if (hipMalloc(&h->d_tab, sizeof(aec::DevTables)) != hipSuccess) return bail(AEC_ERR_OOM);
    aec::DevTables tab;
    aec::build_dev_tables(tab);
    if (hipMemcpy(h->d_tab, &tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess) return bail(AEC_ERR_HIP);
    h->persist = AEC_MODE_KNOB("AEC_CRN_PERSIST", h->persist) != 0;
    h->mx8_shadow = AEC_MODE_KNOB("AEC_CRN_MX8_SHADOW", h->mx8_shadow) != 0;
    if (hipDeviceGetAttribute(&h->num_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) h->num_cus = 0;
    if (h->es == 2 && crn::persist_supported(h->H, h->CELLS, h->S, h->num_cus)) {
        // team arrival counters + error word, and a pinned copy of the error word
        if (hipMalloc(reinterpret_cast<void**>(&h->psync), crn::kPersistSyncInts * sizeof(int)) != hipSuccess)
            return bail(AEC_ERR_OOM);
        if (hipHostMalloc(reinterpret_cast<void**>(&h->perr_host), sizeof(int)) != hipSuccess) return bail(AEC_ERR_OOM);
        *h->perr_host = 0;
        if (hipEventCreateWithFlags(&h->perr_ev, hipEventDisableTiming) != hipSuccess) return bail(AEC_ERR_HIP);
    }
    h->enc.assign(h->L, Packed{});
    h->dec.assign(2 * h->L, Packed{});
    h->decf.assign(h->L, Packed{});
    h->dec_fuse_max = AEC_AB_KNOB("CRN_DEC_FUSE", h->dec_fuse_max);
    h->lih.assign(h->nrnn, Packed{});
    h->lcat.assign(h->nrnn, Packed{});
    h->lhh.assign(h->nrnn, Packed{});
    if (params) {
        const aec_status s = load_params(h, params, n);
        if (s != AEC_OK) return bail(s);
    }
    *out = h;
    return AEC_OK;
}

aec_status aec_crn_set_params(aec_crn_handle* h, const float* params, size_t n) {
    if (!h || !params) return AEC_ERR_INVALID_ARG;
    aec::DeviceGuard dg(h->device);   // the caller's current device is restored on return
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    return load_params(h, params, n);
}

static aec_status prepare(aec_crn_handle* h, const int64_t* lengths, int32_t B, int64_t ld, int64_t* Tmax,
                          hipStream_t st) {
    if (!lengths || B <= 0 || ld <= 0) return crn_fail(h, AEC_ERR_INVALID_ARG, "bad lengths / B / ld");
    int64_t mx = 0;
    for (int b = 0; b < B; ++b) {
        if (lengths[b] < 1 || lengths[b] > ld) return crn_fail(h, AEC_ERR_INVALID_ARG, "length out of [1, ld]");
        mx = std::max(mx, lengths[b]);
    }
    if (mx >= (1ll << 31) / 4) return crn_fail(h, AEC_ERR_INVALID_ARG, "utterance too long");
    *Tmax = mx / 256 + 1;
    aec_status s = ensure_ws(h, B, *Tmax);
    if (s != AEC_OK) return s;
    // the lengths live in the handle (the copy's source outlives the async call);
    // re-uploaded only when they change or the workspace was reallocated
    if (h->last_lens.size() != (size_t)B ||
        !std::equal(lengths, lengths + B, h->last_lens.begin())) {
        h->last_lens.assign(lengths, lengths + B);
        CRN_TRY(h, hipMemcpyAsync(h->d_len, h->last_lens.data(), (size_t)B * sizeof(int64_t), hipMemcpyHostToDevice,
                                  st));
    }
    return AEC_OK;
}

aec_status aec_crn_process(aec_crn_handle* h, const float* mic, const float* far, const int64_t* lengths, int32_t B,
                           int64_t ld, float* out, int64_t ld_out, float* spec, float* mask, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!h->have_params) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameters not set");
    if (!mic || !far) return crn_fail(h, AEC_ERR_INVALID_ARG, "null signal");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    aec::DeviceGuard dg(h->device);   // the caller's current device is restored on return
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    int64_t Tmax = 0;
    aec_status s = prepare(h, lengths, B, ld, &Tmax, st);
    if (s != AEC_OK) return s;
    bool need_out = false;
    for (int b = 0; b < B; ++b) need_out |= lengths[b] >= 256;
    if (need_out && !out) return crn_fail(h, AEC_ERR_INVALID_ARG, "null out");
    int64_t mx = 0;
    for (int b = 0; b < B; ++b) mx = std::max(mx, 256 * (lengths[b] / 256));
    if (out && ld_out < mx) return crn_fail(h, AEC_ERR_INVALID_ARG, "ld_out too small");
    if (h->profile) h->ev_used = 0;
    h->persist_pending = false;
    s = h->es == 4 ? run<float>(h, mic, far, B, ld, Tmax, out, ld_out, spec, mask, st)
                   : run<bf16_t>(h, mic, far, B, ld, Tmax, out, ld_out, spec, mask, st);
    if (s != AEC_OK) {
        h->persist_pending = false;
        return s;
    }
    s = persist_wait(h);                        // a persistent-grid timeout fails this call
    if (s != AEC_OK) return s;
    h->last_B = B;
    h->last_T = Tmax;
    h->proc_lens = h->last_lens;
    if (h->profile && h->ev_used == 6) {
        CRN_TRY(h, hipEventSynchronize(h->ev[5]));
        for (int k = 0; k < 5; ++k) {
            float m = 0.f;
            CRN_TRY(h, hipEventElapsedTime(&m, h->ev[k], h->ev[k + 1]));
            h->ms[k] += m;
        }
        h->calls++;
    }
    return AEC_OK;
}

aec_status aec_crn_stft(aec_crn_handle* h, const float* x, const int64_t* lengths, int32_t B, int64_t ld, float* spec,
                        void* stream) {
    if (!h || !x || !spec) return AEC_ERR_INVALID_ARG;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    aec::DeviceGuard dg(h->device);   // the caller's current device is restored on return
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    int64_t Tmax = 0;
    aec_status s = prepare(h, lengths, B, ld, &Tmax, st);
    if (s != AEC_OK) return s;
    crn::FrontArgs fa{x, x, ld, h->d_len, Tmax, h->d_tab, nullptr, reinterpret_cast<float2*>(spec)};
    CRN_TRY(h, crn::launch_front<float>(fa, B, st));
    return AEC_OK;
}

aec_status aec_crn_error_spec(aec_crn_handle* h, float* spec, void* stream) {
    if (!h || !spec) return AEC_ERR_INVALID_ARG;
    if (h->cfg.nlms_taps <= 0) return crn_fail(h, AEC_ERR_INVALID_ARG, "the handle has no NLMS front end");
    if (h->last_B <= 0) return crn_fail(h, AEC_ERR_INVALID_ARG, "no aec_crn_process call yet");
    aec::DeviceGuard dg(h->device);   // the caller's current device is restored on return
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (h->last_lens != h->proc_lens) {   // an aec_crn_stft since then uploaded other lengths
        h->last_lens = h->proc_lens;
        CRN_TRY(h, hipMemcpyAsync(h->d_len, h->last_lens.data(), h->last_lens.size() * sizeof(int64_t),
                                  hipMemcpyHostToDevice, st));
    }
    CRN_TRY(h, crn::launch_unpack_rows(h->espec, h->d_len, h->last_B, h->last_T, reinterpret_cast<float2*>(spec), st));
    return AEC_OK;
}

aec_status aec_crn_stream_open(aec_crn_handle* h, int32_t B) {
    if (!h || B <= 0) return AEC_ERR_INVALID_ARG;
    if (!h->have_params) return crn_fail(h, AEC_ERR_INVALID_ARG, "parameters not set");
    if (h->nrnn > 8) return crn_fail(h, AEC_ERR_UNSUPPORTED, "too many LSTM layers for streaming");
    aec::DeviceGuard dg(h->device);   // the caller's current device is restored on return
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    stream_free(h);
    h->ss = new (std::nothrow) StreamState();
    if (!h->ss) return AEC_ERR_OOM;
    StreamState& ss = *h->ss;
    ss.B = B;
    const size_t es = h->es;
    const int* ch = h->cfg.conv_channels;
    const int C = h->CELLS, S = h->S, H = h->H;
    auto alloc = [&](void** p, size_t bytes) {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
        if (e == hipSuccess) {
            ss.allocs.push_back(*p);
            e = hipMemset(*p, 0, std::max<size_t>(bytes, 16));
        }
        return e;
    };
    CRN_TRY(h, alloc(&ss.x0, (size_t)B * 256 * 8 * es));
    ss.cat.assign(h->L + 1, nullptr);
    for (int l = 1; l <= h->L; ++l) CRN_TRY(h, alloc(&ss.cat[l], (size_t)B * (256 >> l) * 2 * ch[l] * es));
    CRN_TRY(h, alloc(&ss.gx, (size_t)B * S * C * 4 * H * es));
    if (h->nrnn > 1) CRN_TRY(h, alloc(&ss.xn, (size_t)B * S * H * es));
    if (h->mx8) {
        const size_t qb = (size_t)B * mx8_row_bytes(h);
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.aq), qb));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.as), qb / 32));
    }
    ss.cat8.assign(h->L + 1, nullptr);
    ss.cats.assign(h->L + 1, nullptr);
    for (int l = 1; l <= h->L; ++l)
        if (shadow_level(h, l)) {
            const size_t n8 = (size_t)B * (256 >> l) * 2 * ch[l];
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.cat8[l]), n8));
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.cats[l]), n8 / 32));
        }
    if (shadow_xn(h)) {
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.xn8), (size_t)B * S * H));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.xns), (size_t)B * S * H / 32));
    }
    CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.mask), (size_t)B * 256 * 2 * sizeof(float)));
    if (h->mx8) {
        int64_t skb = 0, skt = 0;
        splitk_need(h, B, &skb, &skt);
        if (skb > 0 && skt <= INT32_MAX) {
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.skp), (size_t)skb));
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.skc), (size_t)skt * sizeof(int)));   // zeroed
            ss.sk_bytes = skb;
            ss.skc_n = (int32_t)skt;
        }
    }
    // dtype 2, NavieComplexLSTM: the recurrence runs as lstm_step_mx8_kernel (AEC_CRN_STEP_MX=0: the bf16
    // step + combine, A/B only)
    const int step_mx = AEC_MODE_KNOB("AEC_CRN_STEP_MX", 1);
    ss.mx_step = step_mx != 0 && h->mx8 && C * S == 4 && h->nrnn > 0 && h->lcat[0].wq != nullptr;
    if (ss.mx_step && h->nrnn > 2) {
        CRN_TRY(h, alloc(&ss.xnb, (size_t)B * S * H * es));
        if (shadow_xn(h)) {
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.xn8b), (size_t)B * S * H));
            CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.xnsb), (size_t)B * S * H / 32));
        }
    }
    if (ss.mx_step) {
        // the kernel's layout preconditions for every layer (x taps of >= 256 k, ...): configs that
        // pass the create-time checks but not these keep the bf16 step + combine
        const Bufs bf{ss.x0,       ss.cat.data(), ss.gx,   ss.xn,  ss.mask,     ss.aq,    ss.as, ss.cat8.data(),
                      ss.cats.data(), ss.xn8,      ss.xns, ss.skp, ss.skc, ss.sk_bytes, ss.skc_n};
        for (int l = 0; l < h->nrnn && ss.mx_step; ++l) {
            crn::StepMxArgs ma;
            mx_step_args(h, ss, bf, l, 0, ma, nullptr);
            ss.mx_step = crn::lstm_step_mx8_layout_ok(ma) && h->lcat[l].wq != nullptr;
        }
    }
    if (ss.mx_step) {
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.hx), (size_t)B * C * S * H * sizeof(float)));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.mx_cnt), (size_t)crn::lstm_step_mx8_counters(H, B) * sizeof(int)));
    }
    for (int l = 0; l < h->nrnn; ++l) {
        if (ss.mx_step) {
            for (int r = 0; r < 2; ++r) {
                CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.ring_q[l][r]), (size_t)B * C * S * H));
                CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.ring_s[l][r]), (size_t)B * C * S * H / 32));
            }
        } else {
            CRN_TRY(h, alloc(&ss.ring_y[l][0], (size_t)B * C * S * H * es));
            CRN_TRY(h, alloc(&ss.ring_y[l][1], (size_t)B * C * S * H * es));
        }
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.cst[l]), (size_t)B * C * S * H * sizeof(float)));
    }
    CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.hop), (size_t)4 * B * 256 * sizeof(float)));
    CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.tail), (size_t)B * 256 * sizeof(float)));
    if (h->cfg.nlms_taps > 0) {
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.nrows), (size_t)B * 512 * sizeof(float2)));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.nstate), (size_t)B * 2 * h->cfg.nlms_taps * 256 * sizeof(float2)));
        CRN_TRY(h, alloc(reinterpret_cast<void**>(&ss.espec), (size_t)B * 256 * sizeof(float2)));
    }
    ss.enc_nlev = stream_enc_levels(h);
    ss.dec_fused = stream_dec_ok(h);
    // the MX folds (one block per stream, 1 wave per SIMD) win while every stream has a CU of its own;
    // past that the unfolded kernels' occupancy (2-3 waves per SIMD) wins: 4,096 streams 4.08 M vs
    // 3.35 M frames/s with both folds, 256 streams 0.1134 vs 0.1204 ms per hop (profiles/r04v_c5_fold_sweep.txt)
    int ncu = 256;
    CRN_TRY(h, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device));
    const bool fold = B <= ncu;
    ss.dec_mx = fold && ss.dec_fused && stream_dec_mx_ok(h);
    ss.enc_mx = fold && ss.enc_nlev == 4 && stream_enc_mx_ok(h);
    CRN_TRY(h, hipStreamCreateWithFlags(&ss.cap, hipStreamNonBlocking));
    CRN_TRY(h, hipDeviceSynchronize());
    ss.k = 0;
    ss.graph_mode = AEC_MODE_KNOB("AEC_CRN_GRAPH", 0) != 0;
    return AEC_OK;
}

static void stream_drop_graphs(StreamState& ss) {
    for (int p = 0; p < 2; ++p) {
        if (ss.graph[p]) (void)hipGraphExecDestroy(ss.graph[p]);
        if (ss.gsrc[p]) (void)hipGraphDestroy(ss.gsrc[p]);
        ss.graph[p] = nullptr;
        ss.gsrc[p] = nullptr;
        ss.front_node[p] = ss.back_node[p] = nullptr;
    }
}

aec_status aec_crn_stream_set_graph(aec_crn_handle* h, int32_t mode) {
    if (!h || !h->ss || mode < 0 || mode > 1) return AEC_ERR_INVALID_ARG;
    aec::DeviceGuard dg(h->device);
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    StreamState& ss = *h->ss;
    if (ss.graph_mode != mode) {
        // the instantiated graphs may still be running: they are destroyed after the device drains
        CRN_TRY(h, hipDeviceSynchronize());
        stream_drop_graphs(ss);
        ss.graph_mode = mode;
    }
    return AEC_OK;
}

aec_status aec_crn_stream_stats(const aec_crn_handle* h, int32_t* graph_mode, int64_t* graph_replays,
                                int64_t* direct_hops) {
    if (!h || !h->ss) return AEC_ERR_INVALID_ARG;
    if (graph_mode) *graph_mode = h->ss->graph_mode;
    if (graph_replays) *graph_replays = h->ss->graph_replays;
    if (direct_hops) *direct_hops = h->ss->direct_hops;
    return AEC_OK;
}

aec_status aec_crn_stream_reset(aec_crn_handle* h, int32_t b, void* stream) {
    if (!h || !h->ss) return AEC_ERR_INVALID_ARG;
    StreamState& ss = *h->ss;
    if (b < -1 || b >= ss.B) return crn_fail(h, AEC_ERR_INVALID_ARG, "stream index out of range");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t es = h->es;
    const size_t hrow = (size_t)h->CELLS * h->S * h->H;       // elements of one stream's h / c rows
    const int b0 = b < 0 ? 0 : b, nb = b < 0 ? ss.B : 1;
    for (int l = 0; l < h->nrnn; ++l) {
        for (int r = 0; r < 2; ++r) {
            if (ss.mx_step) {
                CRN_TRY(h, hipMemsetAsync(ss.ring_q[l][r] + b0 * hrow, 0, nb * hrow, st));
                CRN_TRY(h, hipMemsetAsync(ss.ring_s[l][r] + b0 * hrow / 32, 0, nb * hrow / 32, st));
            } else {
                CRN_TRY(h, hipMemsetAsync(reinterpret_cast<char*>(ss.ring_y[l][r]) + b0 * hrow * es, 0, nb * hrow * es, st));
            }
        }
        CRN_TRY(h, hipMemsetAsync(ss.cst[l] + b0 * hrow, 0, nb * hrow * sizeof(float), st));
    }
    for (int q = 0; q < 4; ++q)
        CRN_TRY(h, hipMemsetAsync(ss.hop + ((size_t)q * ss.B + b0) * 256, 0, (size_t)nb * 256 * sizeof(float), st));
    CRN_TRY(h, hipMemsetAsync(ss.tail + (size_t)b0 * 256, 0, (size_t)nb * 256 * sizeof(float), st));
    if (ss.nstate) {   // NLMS: W, history, P = 0 (a fresh recursion)
        const size_t srow = (size_t)2 * h->cfg.nlms_taps * 256;
        CRN_TRY(h, hipMemsetAsync(ss.nstate + b0 * srow, 0, nb * srow * sizeof(float2), st));
    }
    if (b < 0) ss.k = 0;
    return AEC_OK;
}

aec_status aec_crn_stream_step(aec_crn_handle* h, const float* mic, const float* far, int64_t ld_in, float* out,
                               int64_t ld_out, void* stream) {
    if (!h || !h->ss) return AEC_ERR_INVALID_ARG;
    if (!mic || !far || !out || ld_in < 256 || ld_out < 256) return crn_fail(h, AEC_ERR_INVALID_ARG, "bad hop buffers");
    StreamState& ss = *h->ss;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    aec::DeviceGuard dg(h->device);   // the caller's current device is restored on return
    if (dg.err != hipSuccess) return crn_fail(h, AEC_ERR_HIP, "hipSetDevice failed");
    const int par = (int)(ss.k & 1);
    const StreamIo io{mic, far, ld_in, out, ld_out};
    // two per-hop modes, chosen per handle (aec_crn_stream_set_graph; AEC_CRN_GRAPH at stream_open):
    // direct launches (default) or the hop's launches captured once per ring parity in a hipGraph
    // and replayed.  The 7 kernels of a hop run back to back either way; ~8 us pass between two
    // graph replays, more than the direct launches' gaps (profiles/r05_notes.md r05x/r05y).  A
    // graph that cannot be captured or instantiated fails the call: no silent fallback.
    if (ss.graph_mode) {
        if (!ss.graph[par]) {
            hipGraph_t g = nullptr;
            hipError_t e = hipStreamBeginCapture(ss.cap, hipStreamCaptureModeThreadLocal);
            if (e != hipSuccess) return crn_fail(h, AEC_ERR_HIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(e));
            const aec_status s = h->es == 4 ? stream_launches<float>(h, par, io, ss.cap)
                                            : stream_launches<bf16_t>(h, par, io, ss.cap);
            e = hipStreamEndCapture(ss.cap, &g);
            (void)hipGetLastError();
            std::string why;
            if (s != AEC_OK) why = "a launch failed under capture: " + h->err;
            else if (e != hipSuccess || !g) why = std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
            else if (!ss.front_node[par] || !ss.back_node[par]) why = "the front / back kernel nodes were not captured";
            else if ((e = hipGraphInstantiate(&ss.graph[par], g, nullptr, nullptr, 0)) != hipSuccess)
                why = std::string("hipGraphInstantiate: ") + hipGetErrorString(e);
            if (!why.empty()) {
                if (g) (void)hipGraphDestroy(g);
                ss.graph[par] = nullptr;
                ss.front_node[par] = ss.back_node[par] = nullptr;
                return crn_fail(h, AEC_ERR_HIP, "graph mode: " + why);
            }
            ss.gsrc[par] = g;                          // the node handles belong to it
        } else {
            const aec_status s = stream_set_io(h, par, io);
            if (s != AEC_OK) return s;
        }
        CRN_TRY(h, hipGraphLaunch(ss.graph[par], st));
        ss.graph_replays++;
    } else {
        const aec_status s = h->es == 4 ? stream_launches<float>(h, par, io, st) : stream_launches<bf16_t>(h, par, io, st);
        if (s != AEC_OK) return s;
        ss.direct_hops++;
    }
    ss.k++;
    return AEC_OK;
}

aec_status aec_crn_profile_enable(aec_crn_handle* h, int32_t enable) {
    if (!h) return AEC_ERR_INVALID_ARG;
    h->profile = enable != 0;
    return AEC_OK;
}

aec_status aec_crn_profile_read(aec_crn_handle* h, double* ms5, int64_t* calls) {
    if (!h || !ms5) return AEC_ERR_INVALID_ARG;
    for (int k = 0; k < 5; ++k) {
        ms5[k] = h->ms[k];
        h->ms[k] = 0;
    }
    if (calls) *calls = h->calls;
    h->calls = 0;
    return AEC_OK;
}

void aec_crn_destroy(aec_crn_handle* h) {
    if (!h) return;
    aec::DeviceGuard dg(h->device);
    stream_free(h);
    for (void* p : h->allocs) (void)hipFree(p);
    for (auto* v : {&h->enc, &h->dec, &h->decf, &h->lih, &h->lhh, &h->lcat})
        for (Packed& pk : *v) {
            if (pk.w) (void)hipFree(pk.w);
            if (pk.bias) (void)hipFree(pk.bias);
            if (pk.wq) (void)hipFree(pk.wq);
            if (pk.wsc) (void)hipFree(pk.wsc);
        }
    if (h->d_tab) (void)hipFree(h->d_tab);
    if (h->perr_ev) (void)hipEventDestroy(h->perr_ev);
    if (h->psync) (void)hipFree(h->psync);
    if (h->perr_host) (void)hipHostFree(h->perr_host);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    delete h;
}

}  // extern "C"
