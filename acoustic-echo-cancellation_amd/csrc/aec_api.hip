// aec_api.hip — the C ABI (include/aec_hip.h) over the gfx950 kernels.
//
// Replaces the reference's Little_net construction / load_state_dict /
// forward (Stage2_lhm/scripts/network/ERB.py:203-334, scripts/test.py:102-157).
// The handle owns device copies of the weights, the ERB sparse tables, the
// STFT constant tables and a grow-only workspace; the caller owns all I/O.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/aec_hip.h"
#include "aec_launch.h"
#include "aec_tables.h"

using namespace aec;

struct aec_handle {
    aec_config cfg{};
    int device = 0;
    std::string err;
    float* d_w = nullptr;        // weights blob
    DevTables* d_tab = nullptr;
    int* d_erb = nullptr;        // ErbCSR blob
    int nnz = 0;
    bool have_w = false, have_erb = false;
    // workspace (grow-only)
    int64_t ws_B = 0, ws_T = 0;
    float* d_c = nullptr;        // [B][3]
    int64_t* d_len = nullptr;    // [B]
    float* d_feats = nullptr;    // [B][T][96]
    float* d_est = nullptr;      // [B][T][32]
    float* d_dbg = nullptr;      // [2][B][T][32]  (h, mask)
    std::vector<int64_t> last_lens;
    int debug = 0;
    int64_t last_B = 0, last_T = 0;
    // kernel timing (aec_profile_*)
    int profile = 0;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
};

static hipEvent_t next_event(aec_handle* h) {
    if (h->ev_used == h->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        h->ev_pool.push_back(e);
    }
    return h->ev_pool[h->ev_used++];
}
static void mark(aec_handle* h, hipStream_t st) {
    if (!h->profile) return;
    hipEvent_t e = next_event(h);
    if (e) (void)hipEventRecord(e, st);
}

static const size_t kWeights32 = 96 * 64 + 96 * 32 + 96 + 96 + 32 * 64 + 32 + 32 * 32 + 32;

#define HIP_TRY(h, expr)                                                                 \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            (h)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                \
            return e_ == hipErrorOutOfMemory ? AEC_ERR_OOM : AEC_ERR_HIP;                \
        }                                                                                \
    } while (0)

static aec_status fail(aec_handle* h, aec_status s, const std::string& m) {
    if (h) h->err = m;
    return s;
}

extern "C" {

size_t aec_weights_count(int32_t erb_bands) { return erb_bands == 32 ? kWeights32 : 0; }
int64_t aec_num_frames(int64_t n) { return n / 256 + 1; }
int64_t aec_out_len(int64_t n) { return 256 * (n / 256); }

const char* aec_last_error(const aec_handle* h) { return h ? h->err.c_str() : "null handle"; }

static void build_tables(DevTables& t) {
    const double PI = 3.14159265358979323846;
    for (int j = 0; j < 256; ++j) t.tw256[j] = make_float2((float)std::cos(2 * PI * j / 256), (float)-std::sin(2 * PI * j / 256));
    for (int k = 0; k < 258; ++k) t.tw512[k] = make_float2((float)std::cos(2 * PI * k / 512), (float)-std::sin(2 * PI * k / 512));
    for (int n = 0; n < 512; ++n) t.hann[n] = (float)(0.5 - 0.5 * std::cos(2 * PI * n / 512));
    for (int r = 0; r < 256; ++r) {
        const float a = t.hann[r], b = t.hann[r + 256];
        const float c = a * a + b * b;      // f32, as conv_transpose1d(window^2, eye) does
        t.coffp[r] = c + 1e-8f;
    }
}

aec_status aec_set_weights(aec_handle* h, const float* w, size_t n) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!w || n != kWeights32) return fail(h, AEC_ERR_INVALID_ARG, "weights blob must hold 12544 floats");
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipMemcpy(h->d_w, w, n * sizeof(float), hipMemcpyHostToDevice));
    h->have_w = true;
    return AEC_OK;
}

aec_status aec_set_erb(aec_handle* h, const float* erb) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!erb) return fail(h, AEC_ERR_INVALID_ARG, "erb matrix is null");
    const int NB = 32, NF = 257;
    std::vector<int> band_ptr(NB + 1, 0), bin_ptr(NF + 1, 0), band_bin, bin_band;
    std::vector<float> band_w, bin_w;
    for (int j = 0; j < NB; ++j) {
        band_ptr[j] = (int)band_bin.size();
        for (int k = 0; k < NF; ++k) {
            const float v = erb[k * NB + j];
            if (v != 0.f) { band_bin.push_back(k); band_w.push_back(v); }
        }
    }
    band_ptr[NB] = (int)band_bin.size();
    for (int k = 0; k < NF; ++k) {
        bin_ptr[k] = (int)bin_band.size();
        for (int j = 0; j < NB; ++j) {
            const float v = erb[k * NB + j];
            if (v != 0.f) { bin_band.push_back(j); bin_w.push_back(v); }
        }
    }
    bin_ptr[NF] = (int)bin_band.size();
    const int nnz = (int)band_bin.size();
    if (nnz > 2048) return fail(h, AEC_ERR_UNSUPPORTED, "erb matrix has > 2048 non-zeros (banded filterbanks only)");
    std::vector<int> blob(erb_blob_words(nnz), 0);
    std::memcpy(blob.data(), band_ptr.data(), 33 * 4);
    std::memcpy(blob.data() + 33, bin_ptr.data(), 258 * 4);
    std::memcpy(blob.data() + 33 + 258, band_bin.data(), nnz * 4);
    std::memcpy(blob.data() + 33 + 258 + nnz, band_w.data(), nnz * 4);
    std::memcpy(blob.data() + 33 + 258 + 2 * nnz, bin_band.data(), nnz * 4);
    std::memcpy(blob.data() + 33 + 258 + 3 * nnz, bin_w.data(), nnz * 4);
    HIP_TRY(h, hipSetDevice(h->device));
    if (h->d_erb) { HIP_TRY(h, hipFree(h->d_erb)); h->d_erb = nullptr; }
    HIP_TRY(h, hipMalloc(&h->d_erb, blob.size() * 4));
    HIP_TRY(h, hipMemcpy(h->d_erb, blob.data(), blob.size() * 4, hipMemcpyHostToDevice));
    h->nnz = nnz;
    h->have_erb = true;
    return AEC_OK;
}

aec_status aec_create(const aec_config* cfg, const float* weights, size_t n_weights,
                      const float* erb, int32_t device, aec_handle** out) {
    if (!out) return AEC_ERR_INVALID_ARG;
    *out = nullptr;
    if (!cfg) return AEC_ERR_INVALID_ARG;
    if (cfg->win_size != 512 || cfg->hop_size != 256 || cfg->erb_bands != 32) return AEC_ERR_UNSUPPORTED;
    if (cfg->nlms_taps != 0) return AEC_ERR_UNSUPPORTED;   // FD-NLMS: not in this build yet
    aec_handle* h = new (std::nothrow) aec_handle();
    if (!h) return AEC_ERR_OOM;
    h->cfg = *cfg;
    h->device = device;
    auto bail = [&](aec_status s) { aec_destroy(h); return s; };
    if (hipSetDevice(device) != hipSuccess) return bail(AEC_ERR_HIP);
    if (hipMalloc(&h->d_w, kWeights32 * sizeof(float)) != hipSuccess) return bail(AEC_ERR_OOM);
    if (hipMemset(h->d_w, 0, kWeights32 * sizeof(float)) != hipSuccess) return bail(AEC_ERR_HIP);
    if (hipMalloc(&h->d_tab, sizeof(DevTables)) != hipSuccess) return bail(AEC_ERR_OOM);
    DevTables tab;
    build_tables(tab);
    if (hipMemcpy(h->d_tab, &tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess) return bail(AEC_ERR_HIP);
    if (weights && aec_set_weights(h, weights, n_weights) != AEC_OK) return bail(AEC_ERR_INVALID_ARG);
    if (erb) {
        const aec_status s = aec_set_erb(h, erb);
        if (s != AEC_OK) return bail(s);
    }
    *out = h;
    return AEC_OK;
}

static aec_status ensure_ws(aec_handle* h, int64_t B, int64_t T) {
    if (B <= h->ws_B && T <= h->ws_T) return AEC_OK;
    const int64_t nB = B > h->ws_B ? B : h->ws_B;
    const int64_t nT = T > h->ws_T ? T : h->ws_T;
    HIP_TRY(h, hipDeviceSynchronize());
    (void)hipFree(h->d_c); (void)hipFree(h->d_len); (void)hipFree(h->d_feats); (void)hipFree(h->d_est); (void)hipFree(h->d_dbg);
    h->d_c = nullptr; h->d_len = nullptr; h->d_feats = h->d_est = h->d_dbg = nullptr;
    h->ws_B = h->ws_T = 0;
    h->last_lens.clear();
    HIP_TRY(h, hipMalloc(&h->d_c, nB * 3 * sizeof(float)));
    HIP_TRY(h, hipMalloc(&h->d_len, nB * sizeof(int64_t)));
    HIP_TRY(h, hipMalloc(&h->d_feats, nB * nT * 96 * sizeof(float)));
    HIP_TRY(h, hipMalloc(&h->d_est, nB * nT * 32 * sizeof(float)));
    HIP_TRY(h, hipMalloc(&h->d_dbg, 2 * nB * nT * 32 * sizeof(float)));
    h->ws_B = nB;
    h->ws_T = nT;
    return AEC_OK;
}

aec_status aec_set_debug(aec_handle* h, int32_t enable) {
    if (!h) return AEC_ERR_INVALID_ARG;
    h->debug = enable != 0;
    return AEC_OK;
}

aec_status aec_process(aec_handle* h, const float* mic, const float* ref, const float* near,
                       const int64_t* lengths, int32_t B, int64_t ld, float* out, int64_t ld_out,
                       float* loss, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!h->have_w || !h->have_erb) return fail(h, AEC_ERR_INVALID_ARG, "weights / erb not set");
    if (B < 0 || !lengths) return fail(h, AEC_ERR_INVALID_ARG, "bad batch / lengths");
    if (B == 0) return AEC_OK;
    if (!mic || !ref || !out) return fail(h, AEC_ERR_INVALID_ARG, "null mic / ref / out");
    if (loss && !near) return fail(h, AEC_ERR_INVALID_ARG, "loss requires near");
    int64_t nmax = 0;
    for (int b = 0; b < B; ++b) {
        if (lengths[b] < 1 || lengths[b] > ld) return fail(h, AEC_ERR_INVALID_ARG, "length out of [1, ld]");
        if (aec_out_len(lengths[b]) > ld_out) return fail(h, AEC_ERR_INVALID_ARG, "ld_out too small");
        nmax = lengths[b] > nmax ? lengths[b] : nmax;
    }
    const int64_t Tmax = aec_num_frames(nmax);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    HIP_TRY(h, hipSetDevice(h->device));
    aec_status s = ensure_ws(h, B, Tmax);
    if (s != AEC_OK) return s;
    if (h->last_lens.size() != (size_t)B || std::memcmp(h->last_lens.data(), lengths, B * sizeof(int64_t)) != 0) {
        h->last_lens.assign(lengths, lengths + B);
        // pageable source: staged synchronously by the runtime, safe to reuse on return
        HIP_TRY(h, hipMemcpyAsync(h->d_len, h->last_lens.data(), B * sizeof(int64_t), hipMemcpyHostToDevice, st));
    }
    const int nsig = near ? 3 : 2;
    mark(h, st);
    HIP_TRY(h, launch_moments(mic, ref, near, ld, h->d_len, h->d_c, B, nsig, st));

    AnalysisArgs a{};
    a.sig[0] = mic; a.sig[1] = ref; a.sig[2] = near;
    a.ld = ld; a.lens = h->d_len; a.cvals = h->d_c;
    a.tables = reinterpret_cast<const float*>(h->d_tab);
    a.erb_csr = h->d_erb; a.nnz = h->nnz; a.nsig = nsig;
    a.feats = h->d_feats; a.Tmax = Tmax;
    mark(h, st);
    HIP_TRY(h, launch_analysis(a, B, st));
    mark(h, st);

    GruArgs g{};
    g.feats = h->d_feats; g.Tmax = Tmax; g.lens = h->d_len; g.w = h->d_w;
    g.est = h->d_est; g.loss = loss; g.has_near = near != nullptr;
    g.dbg_h = h->debug ? h->d_dbg : nullptr;
    g.dbg_mask = h->debug ? h->d_dbg + B * Tmax * 32 : nullptr;
    HIP_TRY(h, launch_gru(g, B, st));
    mark(h, st);

    SynthArgs y{};
    y.mic = mic; y.ld = ld; y.lens = h->d_len; y.cvals = h->d_c;
    y.tables = reinterpret_cast<const float*>(h->d_tab);
    y.erb_csr = h->d_erb; y.nnz = h->nnz; y.est = h->d_est; y.Tmax = Tmax;
    y.out = out; y.ld_out = ld_out;
    HIP_TRY(h, launch_synthesis(y, B, st));
    mark(h, st);
    h->last_B = B;
    h->last_T = Tmax;
    return AEC_OK;
}

aec_status aec_debug_copy(aec_handle* h, int32_t what, float* dst, size_t n, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    const int64_t B = h->last_B, T = h->last_T;
    if (!dst || n < (size_t)(B * T * 32)) return fail(h, AEC_ERR_INVALID_ARG, "dst too small");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    HIP_TRY(h, hipSetDevice(h->device));
    if (what >= 0 && what <= 2) {
        HIP_TRY(h, hipMemcpy2DAsync(dst, 32 * sizeof(float), h->d_feats + 32 * what, 96 * sizeof(float),
                                    32 * sizeof(float), B * T, hipMemcpyDeviceToDevice, st));
    } else if (what == 3 || what == 4) {
        if (!h->debug) return fail(h, AEC_ERR_INVALID_ARG, "enable aec_set_debug before aec_process");
        HIP_TRY(h, hipMemcpyAsync(dst, h->d_dbg + (what - 3) * B * T * 32, B * T * 32 * sizeof(float),
                                  hipMemcpyDeviceToDevice, st));
    } else if (what == 5) {
        HIP_TRY(h, hipMemcpyAsync(dst, h->d_est, B * T * 32 * sizeof(float), hipMemcpyDeviceToDevice, st));
    } else {
        return fail(h, AEC_ERR_INVALID_ARG, "unknown intermediate");
    }
    return AEC_OK;
}

aec_status aec_profile_enable(aec_handle* h, int32_t enable) {
    if (!h) return AEC_ERR_INVALID_ARG;
    h->profile = enable != 0;
    h->ev_used = 0;
    return AEC_OK;
}

aec_status aec_profile_read(aec_handle* h, double* ms4, int64_t* calls) {
    if (!h || !ms4) return AEC_ERR_INVALID_ARG;
    for (int i = 0; i < 4; ++i) ms4[i] = 0.0;
    // marks per call: before moments, after moments, after analysis, after gru, after synthesis
    const size_t per = 5;
    const size_t n = h->ev_used / per;
    for (size_t c = 0; c < n; ++c) {
        hipEvent_t* e = &h->ev_pool[c * per];
        HIP_TRY(h, hipEventSynchronize(e[per - 1]));
        for (int k = 0; k < 4; ++k) {
            float ms = 0.f;
            HIP_TRY(h, hipEventElapsedTime(&ms, e[k], e[k + 1]));
            ms4[k] += ms;
        }
    }
    if (calls) *calls = (int64_t)n;
    h->ev_used = 0;
    return AEC_OK;
}

void aec_destroy(aec_handle* h) {
    if (!h) return;
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    (void)hipSetDevice(h->device);
    (void)hipFree(h->d_w); (void)hipFree(h->d_tab); (void)hipFree(h->d_erb);
    (void)hipFree(h->d_c); (void)hipFree(h->d_len); (void)hipFree(h->d_feats); (void)hipFree(h->d_est); (void)hipFree(h->d_dbg);
    delete h;
}

}  // extern "C"
