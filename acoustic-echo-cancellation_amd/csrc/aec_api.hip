// aec_api.hip — the C ABI (include/aec_hip.h) over the gfx950 kernels.
//
// Replaces the reference's Little_net construction / load_state_dict /
// forward (Stage2_lhm/scripts/network/ERB.py:203-334, scripts/test.py:102-157).
// The handle owns device copies of the weights, the ERB sparse tables, the
// STFT constant tables and a grow-only workspace; the caller owns all I/O.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/aec_hip.h"
#include "aec_device.h"
#include "aec_launch.h"
#include "aec_tables.h"


// ---------------------------------------------------------------------------
// ERB tables (see aec_tables.h): balanced forward schedule + transpose table
// ---------------------------------------------------------------------------
namespace aec {
ErbTables build_erb_tables(const float* erb) {
    const int NB = 32, NF = 257, LANES = 16, SLOTS = 3;
    ErbTables t;
    std::vector<std::vector<int>> bins(NB);
    int maxw = 0, nnz = 0;
    for (int j = 0; j < NB; ++j) {
        for (int k = 0; k < NF; ++k)
            if (erb[k * NB + j] != 0.f) bins[j].push_back(k);
        maxw = std::max(maxw, (int)bins[j].size());
        nnz += (int)bins[j].size();
    }
    // transpose table: <= 2 bands per bin
    t.bintab.assign(NF * 4, 0.f);
    for (int k = 0; k < NF; ++k) {
        int cnt = 0;
        for (int j = 0; j < NB; ++j) {
            const float v = erb[k * NB + j];
            if (v == 0.f) continue;
            if (cnt == 2) { t.why = "a bin lies in more than 2 bands"; return t; }
            int ib = j;
            std::memcpy(&t.bintab[k * 4 + 2 * cnt], &ib, 4);
            t.bintab[k * 4 + 2 * cnt + 1] = v;
            ++cnt;
        }
        if (cnt == 1) { int ib; std::memcpy(&ib, &t.bintab[k * 4], 4); std::memcpy(&t.bintab[k * 4 + 2], &ib, 4); }
    }
    // forward schedule: split bands wider than `split` in two, pack pieces
    struct Piece { int band, first, count; };
    for (int split = std::max(26, (maxw + 1) / 2); split <= NF; split += 2) {
        std::vector<Piece> pieces;
        for (int j = 0; j < NB; ++j) {
            const int w = (int)bins[j].size();
            if (w == 0) continue;
            if (w > split) {
                pieces.push_back({j, 0, (w + 1) / 2});
                pieces.push_back({j, (w + 1) / 2, w - (w + 1) / 2});
            } else {
                pieces.push_back({j, 0, w});
            }
        }
        std::stable_sort(pieces.begin(), pieces.end(), [](const Piece& a, const Piece& b) { return a.count > b.count; });
        std::vector<std::vector<int>> lane(LANES);
        std::vector<int> load(LANES, 0);
        bool fits = true;
        for (int p = 0; p < (int)pieces.size() && fits; ++p) {
            int best = -1;
            for (int l = 0; l < LANES; ++l)
                if ((int)lane[l].size() < SLOTS && (best < 0 || load[l] < load[best])) best = l;
            if (best < 0) fits = false;
            else { lane[best].push_back(p); load[best] += pieces[p].count; }
        }
        if (!fits) continue;
        int L = 0;
        for (int l = 0; l < LANES; ++l) L = std::max(L, load[l]);
        L = (L + 3) & ~3;
        if (L > 48) { t.why = "ERB schedule longer than 48 entries per lane"; return t; }
        t.sched_len = L;
        t.sched.assign((size_t)L * LANES * 4 + 64, 0.f);
        std::vector<int> comb(2 * NB, -1);
        // Order every lane's entries so that at each step the 16 lanes read
        // bins with distinct residues mod 16: with the per-frame XOR swizzle the
        // 32 lanes of a ds_read_b32 then hit 32 distinct banks.  One bipartite
        // matching (lanes x residues, Kuhn) per step; lanes with no slack left
        // must take a real entry, the others may take a zero-weight padding
        // entry on a free residue (bin = residue).
        struct Item { int k, s; float w; };
        std::vector<std::vector<Item>> items(LANES);
        for (int l = 0; l < LANES; ++l)
            for (int s = 0; s < (int)lane[l].size(); ++s) {
                const Piece& pc = pieces[lane[l][s]];
                for (int i = 0; i < pc.count; ++i) {
                    const int k = bins[pc.band][pc.first + i];
                    items[l].push_back({k, s, erb[k * NB + pc.band]});
                }
                const int slot = 3 * l + s;
                if (comb[2 * pc.band] < 0) comb[2 * pc.band] = slot;
                else comb[2 * pc.band + 1] = slot;
            }
        t.conflicts = 0;
        for (int e = 0; e < L; ++e) {
            const int left = L - e;
            std::vector<int> owner(16, -1), match(LANES, -1);
            std::vector<int> order(LANES);
            for (int l = 0; l < LANES; ++l) order[l] = l;
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
                return left - (int)items[a].size() < left - (int)items[b].size(); });
            std::function<bool(int, std::vector<char>&)> aug = [&](int l, std::vector<char>& seen) -> bool {
                for (const Item& it : items[l]) {
                    const int r = it.k & 15;
                    if (seen[r]) continue;
                    seen[r] = 1;
                    if (owner[r] < 0 || aug(owner[r], seen)) { owner[r] = l; match[l] = r; return true; }
                }
                return false;
            };
            for (int l : order) {
                if (items[l].empty()) continue;
                std::vector<char> seen(16, 0);
                aug(l, seen);
            }
            for (int l = 0; l < LANES; ++l) {
                float* en = &t.sched[((size_t)e * LANES + l) * 4];
                if (match[l] >= 0) {
                    for (size_t i = 0; i < items[l].size(); ++i)
                        if ((items[l][i].k & 15) == match[l]) {
                            const Item it = items[l][i];
                            std::memcpy(&en[0], &it.k, 4);
                            en[1 + it.s] = it.w;
                            items[l].erase(items[l].begin() + i);
                            break;
                        }
                } else if ((int)items[l].size() >= left) {       // no slack: take one anyway
                    const Item it = items[l].front();
                    std::memcpy(&en[0], &it.k, 4);
                    en[1 + it.s] = it.w;
                    items[l].erase(items[l].begin());
                    ++t.conflicts;
                } else {                                          // zero-weight padding on a free residue
                    int r = 0;
                    while (owner[r] >= 0) ++r;
                    owner[r] = l;
                    std::memcpy(&en[0], &r, 4);
                }
            }
        }
        // bands with no non-zeros read a zero slot: point both at a lane with < 3 pieces, else -1 pair
        for (int j = 0; j < NB; ++j) {
            if (comb[2 * j] < 0) {
                int z = -1;
                for (int l = 0; l < LANES && z < 0; ++l)
                    if ((int)lane[l].size() < SLOTS) z = 3 * l + (int)lane[l].size();
                if (z < 0) { t.why = "no zero slot for an empty band"; return t; }
                comb[2 * j] = z;
            }
        }
        std::memcpy(&t.sched[(size_t)L * LANES * 4], comb.data(), 64 * 4);
        t.ok = true;
        return t;
    }
    t.why = "could not balance the ERB schedule";
    return t;
}
}  // namespace aec

using namespace aec;

struct aec_handle {
    aec_config cfg{};
    int device = 0;
    std::string err;
    float* d_w = nullptr;        // weights blob
    DevTables* d_tab = nullptr;
    float* d_sched = nullptr;    // ERB forward schedule (ErbTables::sched)
    float* d_bintab = nullptr;   // ERB transpose table (ErbTables::bintab)
    int sched_len = 0;
    bool have_w = false, have_erb = false;
    // workspace (grow-only)
    int64_t ws_B = 0, ws_T = 0;
    double2* d_mom = nullptr;    // [B][3][kMomChunks]
    float* d_cvals = nullptr;    // [B][3]
    // work lists of the last batch shape (prepare_lists): one device block
    // [items | sitems | len | slen] rewritten in stream order from a ring of two
    // pinned host slots; no device-wide synchronisation when the lengths change
    char* d_lists = nullptr;
    size_t lists_cap = 0;
    WorkItem* d_items = nullptr; // analysis work list (4-frame items)
    WorkItem* d_sitems = nullptr; // synthesis block-item list (15 hops)
    int64_t* d_len = nullptr;    // [B] mic length: sets the frame count and output length
    int32_t* d_slen = nullptr;   // [B][4] per-signal lengths (mic, ref, near, -): normaliser + zero padding
    int64_t nitems = 0, nsitems = 0;
    // look-ahead normaliser passes (aec_prepare_siglens), consumed in order by the process calls
    struct PreSlot {
        double2* mom = nullptr;       // [cap][3][kMomChunks]
        float* cvals = nullptr;       // [cap][3]
        int32_t* slen = nullptr;      // device [cap][4]
        int32_t* host = nullptr;      // pinned [cap][4] (upload staging)
        int64_t cap = 0;
        hipEvent_t done = nullptr;    // recorded after norm_finalize on the prepare stream
        hipEvent_t freed = nullptr;   // recorded after the consuming call's kernels
        bool used = false;            // done / freed recorded at least once
        bool freed_rec = false;
        const float* sig[3] = {nullptr, nullptr, nullptr};
        int64_t ld = 0;
        int nsig = 0;
        std::vector<int64_t> l3;
        uint64_t token = 0;
    };
    PreSlot pre[2];
    int pre_head = 0, pre_count = 0;
    uint64_t next_token = 1;
    struct ListSlot {
        char* host = nullptr;    // pinned
        size_t cap = 0;
        hipEvent_t ev = nullptr; // recorded after the upload from this slot
        bool pending = false;
    };
    ListSlot slots[2];
    int slot_next = 0;
    int last_nsig = 0;
    int num_cus = 256;
    std::vector<int64_t> item_off, sitem_off;   // first analysis / synthesis item of stream b (B+1 entries)
    // ordering of this handle's calls: a call on another stream than the last one
    // waits (on the device) for the last one, since they share the workspace
    hipEvent_t ev_last = nullptr;
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    float* d_feats = nullptr;    // [B][T][96]
    float* d_est = nullptr;      // [B][T][32]
    float* d_dbg = nullptr;      // [2][B][T][32]  (h, mask)
    float2* d_spec = nullptr;    // [B][T][256] NLMS error spectrum (nlms_taps > 0 only)
    std::vector<int64_t> last_lens;                 // [B][3] of the last call (work lists rebuilt on change)
    std::vector<WorkItem> h_items, h_sitems;        // host copies of the last work lists
    int debug = 0;
    int gru_mode = 0;            // AEC_GRU_MODE (A/B builds: timing experiments; results invalid unless 0)
    int nlms_mode = 0;           // AEC_NLMS_MODE: bit 4 two-pass ref ERB (tested); bits 0-3 A/B builds only (skip work)
    int nlms_prio = 0;           // AEC_NLMS_PRIO (A/B builds): wave priorities mic|ref|nlms digits (0 fastest measured)
    int nlms_erb = 0;            // AEC_NLMS_ERB (A/B builds): role running the mic_erb pass (0: the mic
                                 // waves without a near signal, else the ref waves; 1 ref, 2 nlms)
    int fused = 1;               // AEC_FUSED_SYNTH: GRU + synthesis in one kernel (NLMS path)
    int fused_mode = 0;          // AEC_FUSED_MODE (A/B builds: timing experiments; results invalid unless 0)
    int small_b = -1;            // AEC_SMALLB: NLMS batches up to this many streams take the split path;
                                 // default half the CUs (the pipelined split path's limit).  Against the
                                 // per-stream K2n block, one 10 s call: B = 1 0.258 vs 0.557 ms, 65 0.343
                                 // vs 0.491, 96 0.413 vs 0.505, 128 0.490 vs 0.527 (r06h, r06m)
    float2* d_rows = nullptr;    // split path: packed mic / ref rows [B][T][2][256]
    size_t rows_cap = 0;         // float2 elements
    // split path, pipelined (AEC_SMALLB_PIPE, default on): the recursion and mic_erb run in producer
    // blocks of the GRU + synthesis launch (aec_gru_synth.hip, launch_gru_synth_pipe)
    int small_pipe = 1;
    unsigned long long* d_progress = nullptr;       // [progress_cap] per-stream published chunks
    int progress_cap = 0;
    unsigned long long pipe_epoch = 0;
    int* h_pipe_err = nullptr;   // host-mapped: a consumer wave of an earlier launch stopped waiting
    int* d_pipe_err = nullptr;
    int64_t last_B = 0, last_T = 0;
    // kernel timing (aec_profile_*)
    int profile = 0;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    // streaming (aec_stream_*): per-stream state [stream_B][stream_stride]
    float* d_state = nullptr;
    int32_t stream_B = 0;
    int64_t stream_stride = 0;
    // training (aec_train_*): state of the last aec_train_forward, read by aec_train_backward
    float* d_th = nullptr;       // [B][T][32] GRU outputs
    float* d_tloss = nullptr;    // [B] per-row loss
    float* d_rec = nullptr;      // [B*T][8][32]
    float* d_dg = nullptr;       // [B*T][4][32]
    float* d_part = nullptr;     // [nblk][12544]
    float* d_scan = nullptr;     // chunked-scan BPTT: [B][chunks][32][32 + 2]
    int64_t scan_cap = 0;        // floats d_scan holds
    int bptt_serial = 0;         // AEC_BPTT_SERIAL=1: the one-wave-per-stream BPTT (A/B)
    int64_t train_cap = 0;       // frames the training buffers hold
    int32_t train_rows = 0;      // rows d_tloss holds
    int32_t part_cap = 0;        // blocks d_part holds
    int32_t train_B = 0, train_T = 0;
    int64_t train_gen = 0;       // incremented by every aec_train_forward
};

static hipEvent_t next_event(aec_handle* h) {
    if (h->ev_used == h->ev_pool.size()) {
        hipEvent_t e;
        // timing marks without the system-scope release fence a default event adds
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
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

// select the handle's device for the rest of the entry point; the caller's
// current device is restored on return (aec_device.h)
#define AEC_ON_DEVICE(h)                                                                  \
    DeviceGuard dg_((h)->device);                                                         \
    if (dg_.err != hipSuccess) {                                                          \
        (h)->err = std::string("hipSetDevice: ") + hipGetErrorString(dg_.err);            \
        return AEC_ERR_HIP;                                                               \
    }

static aec_status fail(aec_handle* h, aec_status s, const std::string& m) {
    if (h) h->err = m;
    return s;
}

namespace aec {
// STFT constant tables, float64 math rounded to float32 (aec_tables.h)
void build_dev_tables(DevTables& t) {
    const double PI = 3.14159265358979323846;
    for (int k1 = 0; k1 < 16; ++k1)
        for (int lb = 0; lb < 16; ++lb) {
            const int j = (lb * k1) & 255;
            t.twT[k1 * 16 + lb] = make_float2((float)std::cos(2 * PI * j / 256), (float)-std::sin(2 * PI * j / 256));
        }
    for (int k = 0; k < 258; ++k) t.tw512[k] = make_float2((float)std::cos(2 * PI * k / 512), (float)-std::sin(2 * PI * k / 512));
    for (int n = 0; n < 512; ++n) t.hann[n] = (float)(0.5 - 0.5 * std::cos(2 * PI * n / 512));
    for (int r = 0; r < 256; ++r) {
        const float a = t.hann[r], b = t.hann[r + 256];
        const float c = a * a + b * b;      // f32, as conv_transpose1d(window^2, eye) does
        t.inv_coff[r] = (float)(1.0 / (double)(c + 1e-8f));
    }
}
}  // namespace aec

extern "C" {

size_t aec_weights_count(int32_t erb_bands) { return erb_bands == 32 ? kWeights32 : 0; }
int64_t aec_num_frames(int64_t n) { return n / 256 + 1; }
int64_t aec_out_len(int64_t n) { return 256 * (n / 256); }

const char* aec_last_error(const aec_handle* h) { return h ? h->err.c_str() : "null handle"; }

const char* aec_build_info(void) {
    static const std::string info = std::string("arch=gfx950 ab_knobs=") + (AEC_AB_BUILD ? "on" : "off") +
                                    " mode_knobs=" + aec::kModeKnobs;
    return info.c_str();
}


aec_status aec_set_weights(aec_handle* h, const float* w, size_t n) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!w || n != kWeights32) return fail(h, AEC_ERR_INVALID_ARG, "weights blob must hold 12544 floats");
    AEC_ON_DEVICE(h);
    // kernels launched on any stream may still be reading the old blob
    HIP_TRY(h, hipDeviceSynchronize());
    HIP_TRY(h, hipMemcpy(h->d_w, w, n * sizeof(float), hipMemcpyHostToDevice));
    h->have_w = true;
    return AEC_OK;
}

aec_status aec_set_erb(aec_handle* h, const float* erb) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!erb) return fail(h, AEC_ERR_INVALID_ARG, "erb matrix is null");
    const ErbTables t = build_erb_tables(erb);
    if (!t.ok) return fail(h, AEC_ERR_UNSUPPORTED, std::string("erb matrix: ") + t.why);
    AEC_ON_DEVICE(h);
    HIP_TRY(h, hipDeviceSynchronize());   // the previous tables may still be in use
    if (h->d_sched) { HIP_TRY(h, hipFree(h->d_sched)); h->d_sched = nullptr; }
    if (h->d_bintab) { HIP_TRY(h, hipFree(h->d_bintab)); h->d_bintab = nullptr; }
    HIP_TRY(h, hipMalloc(&h->d_sched, t.sched.size() * 4));
    HIP_TRY(h, hipMemcpy(h->d_sched, t.sched.data(), t.sched.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(h, hipMalloc(&h->d_bintab, t.bintab.size() * 4));
    HIP_TRY(h, hipMemcpy(h->d_bintab, t.bintab.data(), t.bintab.size() * 4, hipMemcpyHostToDevice));
    h->sched_len = t.sched_len;
    h->have_erb = true;
    return AEC_OK;
}

aec_status aec_create(const aec_config* cfg, const float* weights, size_t n_weights,
                      const float* erb, int32_t device, aec_handle** out) {
    if (!out) return AEC_ERR_INVALID_ARG;
    *out = nullptr;
    if (!cfg) return AEC_ERR_INVALID_ARG;
    if (cfg->win_size != 512 || cfg->hop_size != 256 || cfg->erb_bands != 32) return AEC_ERR_UNSUPPORTED;
    if (cfg->nlms_taps < 0 || cfg->nlms_taps > 8) return AEC_ERR_UNSUPPORTED;
    if (cfg->nlms_taps > 0 && !(cfg->nlms_mu >= 0.f && cfg->nlms_mu < 2.f && cfg->nlms_beta >= 0.f &&
                                cfg->nlms_beta < 1.f && cfg->nlms_delta > 0.f && std::isfinite(cfg->nlms_delta)))
        return AEC_ERR_INVALID_ARG;
    aec_handle* h = new (std::nothrow) aec_handle();
    if (!h) return AEC_ERR_OOM;
    h->cfg = *cfg;
    h->device = device;
    // tested modes (aec_knobs.h): the two-pass ERB projection of K2n's ref waves (AEC_NLMS_MODE bit 4),
    // the unfused GRU + synthesis, the small-batch split path, the serial BPTT recursion
    h->nlms_mode = AEC_MODE_KNOB("AEC_NLMS_MODE", 0) & 16;
    h->fused = AEC_MODE_KNOB("AEC_FUSED_SYNTH", h->fused);
    h->small_b = AEC_MODE_KNOB("AEC_SMALLB", h->small_b);
    h->small_pipe = AEC_MODE_KNOB("AEC_SMALLB_PIPE", h->small_pipe);
    h->bptt_serial = AEC_MODE_KNOB("AEC_BPTT_SERIAL", h->bptt_serial);
    // A/B builds only: work-skipping timing bits and role priorities
    h->gru_mode = AEC_AB_KNOB("AEC_GRU_MODE", 0);
    h->nlms_mode |= AEC_AB_KNOB("AEC_NLMS_MODE", 0) & ~16;
    h->nlms_prio = AEC_AB_KNOB("AEC_NLMS_PRIO", 0);
    h->nlms_erb = AEC_AB_KNOB("AEC_NLMS_ERB", h->nlms_erb);
    h->fused_mode = AEC_AB_KNOB("AEC_FUSED_MODE", 0);
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            h->num_cus = cus;
    }
    if (h->small_b < 0) h->small_b = h->num_cus / 2;
    auto bail = [&](aec_status s) { aec_destroy(h); return s; };
    DeviceGuard dg(device);
    if (dg.err != hipSuccess) return bail(AEC_ERR_HIP);
    if (hipEventCreateWithFlags(&h->ev_last, hipEventDisableTiming) != hipSuccess) return bail(AEC_ERR_HIP);
    for (auto& sl : h->slots)
        if (hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) != hipSuccess) return bail(AEC_ERR_HIP);

    if (hipMalloc(&h->d_w, kWeights32 * sizeof(float)) != hipSuccess) return bail(AEC_ERR_OOM);
    if (hipMemset(h->d_w, 0, kWeights32 * sizeof(float)) != hipSuccess) return bail(AEC_ERR_HIP);
    if (hipMalloc(&h->d_tab, sizeof(DevTables)) != hipSuccess) return bail(AEC_ERR_OOM);
    DevTables tab;
    build_dev_tables(tab);
    if (hipMemcpy(h->d_tab, &tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess) return bail(AEC_ERR_HIP);
    if (weights && aec_set_weights(h, weights, n_weights) != AEC_OK) return bail(AEC_ERR_INVALID_ARG);
    if (erb) {
        const aec_status s = aec_set_erb(h, erb);
        if (s != AEC_OK) return bail(s);
    }
    *out = h;
    return AEC_OK;
}

// Grow-only workspace.  Growth (a larger batch or longer streams than any
// call before) frees buffers that kernels of earlier calls on any stream may
// still read, so it synchronises the device; a fixed or shrinking shape never
// does.
static aec_status ensure_ws(aec_handle* h, int64_t B, int64_t T) {
    if (B <= h->ws_B && T <= h->ws_T) return AEC_OK;
    const int64_t nB = B > h->ws_B ? B : h->ws_B;
    const int64_t nT = T > h->ws_T ? T : h->ws_T;
    HIP_TRY(h, hipDeviceSynchronize());
    (void)hipFree(h->d_mom); (void)hipFree(h->d_cvals); (void)hipFree(h->d_feats);
    (void)hipFree(h->d_est); (void)hipFree(h->d_dbg); (void)hipFree(h->d_spec);
    h->d_mom = nullptr; h->d_cvals = nullptr; h->d_feats = h->d_est = h->d_dbg = nullptr;
    h->d_spec = nullptr;
    h->ws_B = h->ws_T = 0;
    HIP_TRY(h, hipMalloc(&h->d_mom, nB * 3 * kMomChunks * sizeof(double2)));
    HIP_TRY(h, hipMalloc(&h->d_cvals, nB * 3 * sizeof(float)));
    HIP_TRY(h, hipMalloc(&h->d_feats, nB * nT * 96 * sizeof(float)));
    HIP_TRY(h, hipMalloc(&h->d_est, nB * nT * 32 * sizeof(float)));
    HIP_TRY(h, hipMalloc(&h->d_dbg, 2 * nB * nT * 32 * sizeof(float)));
    if (h->cfg.nlms_taps > 0) HIP_TRY(h, hipMalloc(&h->d_spec, nB * nT * 256 * sizeof(float2)));
    h->ws_B = nB;
    h->ws_T = nT;
    return AEC_OK;
}

// Host-built work lists of a batch (analysis items of 4 frames, synthesis
// items of 15 hops) and the per-stream lengths; rebuilt only when the lengths
// (or whether near is given) change.  The lists go to the device in stream
// order (one copy from a pinned staging slot): kernels of this handle's earlier
// calls are ordered before it on the same stream, and a call on another stream
// first waits for the last one (begin_call).  The host waits only when it
// reuses a staging slot whose copy (two list changes ago) is still in flight,
// or when the device block must grow.
static size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

static aec_status prepare_lists(aec_handle* h, const int64_t* lengths3, int32_t B, int nsig_in, hipStream_t st) {
    if (h->last_nsig == nsig_in && h->last_lens.size() == (size_t)B * 3 &&
        std::memcmp(h->last_lens.data(), lengths3, (size_t)B * 3 * sizeof(int64_t)) == 0)
        return AEC_OK;
    std::vector<int64_t> lens(B);
    for (int b = 0; b < B; ++b) lens[b] = lengths3[3 * b];
    // analysis work list: 4-frame items of every stream, valid frames only
    std::vector<WorkItem>& items = h->h_items;
    items.clear();
    h->item_off.assign(B + 1, 0);
    for (int b = 0; b < B; ++b) {
        h->item_off[b] = (int64_t)items.size();
        const int64_t T = aec_num_frames(lens[b]);
        for (int64_t wt = 0; wt < T; wt += 4) items.push_back({b, (int32_t)wt, lens[b]});
    }
    h->item_off[B] = (int64_t)items.size();
    // synthesis work list: 15 output hops per block item
    std::vector<WorkItem>& sitems = h->h_sitems;
    sitems.clear();
    h->sitem_off.assign(B + 1, 0);
    for (int b = 0; b < B; ++b) {
        h->sitem_off[b] = (int64_t)sitems.size();
        const int64_t nhop = lens[b] / 256;
        for (int64_t h0 = 0; h0 < nhop; h0 += kHopsOut) sitems.push_back({b, (int32_t)h0, lens[b]});
    }
    h->sitem_off[B] = (int64_t)sitems.size();
    // block layout [items | sitems | len | slen], 16-B aligned pieces
    const size_t o_si = align16(items.size() * sizeof(WorkItem));
    const size_t o_len = o_si + align16(sitems.size() * sizeof(WorkItem));
    const size_t o_slen = o_len + align16((size_t)B * sizeof(int64_t));
    const size_t bytes = o_slen + align16((size_t)B * 4 * sizeof(int32_t));
    if (bytes > h->lists_cap) {
        // earlier kernels of this handle may read the old block: wait for the handle's last call
        if (h->have_last) HIP_TRY(h, hipEventSynchronize(h->ev_last));
        if (h->d_lists) HIP_TRY(h, hipFree(h->d_lists));
        h->d_lists = nullptr;
        h->lists_cap = 0;
        const size_t cap = bytes + bytes / 4;
        HIP_TRY(h, hipMalloc(&h->d_lists, cap));
        h->lists_cap = cap;
    }
    aec_handle::ListSlot& sl = h->slots[h->slot_next];
    h->slot_next ^= 1;
    if (sl.pending) HIP_TRY(h, hipEventSynchronize(sl.ev));   // its previous upload has been read
    sl.pending = false;
    if (bytes > sl.cap) {
        if (sl.host) HIP_TRY(h, hipHostFree(sl.host));
        sl.host = nullptr;
        sl.cap = 0;
        HIP_TRY(h, hipHostMalloc(reinterpret_cast<void**>(&sl.host), bytes + bytes / 4));
        sl.cap = bytes + bytes / 4;
    }
    std::memcpy(sl.host, items.data(), items.size() * sizeof(WorkItem));
    std::memcpy(sl.host + o_si, sitems.data(), sitems.size() * sizeof(WorkItem));
    std::memcpy(sl.host + o_len, lens.data(), (size_t)B * sizeof(int64_t));
    int32_t* slen = reinterpret_cast<int32_t*>(sl.host + o_slen);
    for (int b = 0; b < B; ++b) {
        for (int sg = 0; sg < 3; ++sg) slen[4 * b + sg] = (int32_t)(sg < nsig_in ? lengths3[3 * b + sg] : lens[b]);
        slen[4 * b + 3] = 0;
    }
    HIP_TRY(h, hipMemcpyAsync(h->d_lists, sl.host, bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(h, hipEventRecord(sl.ev, st));
    sl.pending = true;
    h->d_items = reinterpret_cast<WorkItem*>(h->d_lists);
    h->d_sitems = reinterpret_cast<WorkItem*>(h->d_lists + o_si);
    h->d_len = reinterpret_cast<int64_t*>(h->d_lists + o_len);
    h->d_slen = reinterpret_cast<int32_t*>(h->d_lists + o_slen);
    h->nitems = (int64_t)items.size();
    h->nsitems = (int64_t)sitems.size();
    h->last_lens.assign(lengths3, lengths3 + (size_t)B * 3);
    h->last_nsig = nsig_in;
    return AEC_OK;
}

// Every call that reads or writes the handle's workspace: ordered after the
// handle's previous call (a device-side wait when the stream changes), and
// recorded as the handle's last call when it has been queued.
static aec_status begin_call(aec_handle* h, hipStream_t st) {
    if (h->have_last && st != h->last_stream) HIP_TRY(h, hipStreamWaitEvent(st, h->ev_last, 0));
    return AEC_OK;
}
static aec_status end_call(aec_handle* h, hipStream_t st) {
    HIP_TRY(h, hipEventRecord(h->ev_last, st));
    h->last_stream = st;
    h->have_last = true;
    return AEC_OK;
}
// every exit after begin_call records ev_last on the call's stream, early error returns
// included: kernels the call already queued stay ordered before the next call on another stream
struct CallGuard {
    aec_handle* h;
    hipStream_t st;
    bool done = false;
    ~CallGuard() {
        if (!done && hipEventRecord(h->ev_last, st) == hipSuccess) {
            h->last_stream = st;
            h->have_last = true;
        }
    }
    aec_status end() {
        done = true;
        return end_call(h, st);
    }
};

aec_status aec_set_debug(aec_handle* h, int32_t enable) {
    if (!h) return AEC_ERR_INVALID_ARG;
    h->debug = enable != 0;
    return AEC_OK;
}

aec_status aec_process(aec_handle* h, const float* mic, const float* ref, const float* near,
                       const int64_t* lengths, int32_t B, int64_t ld, float* out, int64_t ld_out,
                       float* loss, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (B < 0 || !lengths) return fail(h, AEC_ERR_INVALID_ARG, "bad batch / lengths");
    std::vector<int64_t> l3((size_t)B * 3);
    for (int b = 0; b < B; ++b) l3[3 * b] = l3[3 * b + 1] = l3[3 * b + 2] = lengths[b];
    return aec_process_siglens(h, mic, ref, near, l3.data(), B, ld, out, ld_out, loss, stream);
}

static aec_status process_impl(aec_handle* h, uint64_t token, const float* mic, const float* ref, const float* near,
                               const int64_t* lengths3, int32_t B, int64_t ld, float* out, int64_t ld_out,
                               float* loss, void* stream);

aec_status aec_process_siglens(aec_handle* h, const float* mic, const float* ref, const float* near,
                               const int64_t* lengths3, int32_t B, int64_t ld, float* out, int64_t ld_out,
                               float* loss, void* stream) {
    return process_impl(h, 0, mic, ref, near, lengths3, B, ld, out, ld_out, loss, stream);
}

aec_status aec_process_prepared(aec_handle* h, uint64_t token, const float* mic, const float* ref, const float* near,
                                const int64_t* lengths3, int32_t B, int64_t ld, float* out, int64_t ld_out,
                                float* loss, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (token == 0) return fail(h, AEC_ERR_INVALID_ARG, "look-ahead token 0");
    return process_impl(h, token, mic, ref, near, lengths3, B, ld, out, ld_out, loss, stream);
}

static aec_status process_impl(aec_handle* h, uint64_t token, const float* mic, const float* ref, const float* near,
                               const int64_t* lengths3, int32_t B, int64_t ld, float* out, int64_t ld_out,
                               float* loss, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!h->have_w || !h->have_erb) return fail(h, AEC_ERR_INVALID_ARG, "weights / erb not set");
    if (B < 0 || !lengths3) return fail(h, AEC_ERR_INVALID_ARG, "bad batch / lengths");
    if (B == 0) return AEC_OK;
    if (!mic || !ref) return fail(h, AEC_ERR_INVALID_ARG, "null mic / ref");
    if (loss && !near) return fail(h, AEC_ERR_INVALID_ARG, "loss requires near");
    const int nsig_in = near ? 3 : 2;
    int64_t nmax = 0;
    for (int b = 0; b < B; ++b) {
        const int64_t n = lengths3[3 * b];
        for (int s = 0; s < nsig_in; ++s) {
            const int64_t ns = lengths3[3 * b + s];
            if (ns < 1 || ns > ld) return fail(h, AEC_ERR_INVALID_ARG, "length out of [1, ld]");
            if (ns > INT32_MAX - 4096) return fail(h, AEC_ERR_UNSUPPORTED, "stream longer than 2^31 - 4096 samples");
            // Little_net.forward combines the three signals frame by frame
            // (ERB.py:287-290, 318-323): the reference raises on a frame-count mismatch
            if (ns / 256 != n / 256)
                return fail(h, AEC_ERR_INVALID_ARG, "ref / near frame count differs from mic's (N//256 + 1)");
        }
        if (aec_out_len(n) > ld_out) return fail(h, AEC_ERR_INVALID_ARG, "ld_out too small");
        nmax = n > nmax ? n : nmax;
    }
    if (!out && aec_out_len(nmax) > 0) return fail(h, AEC_ERR_INVALID_ARG, "null out");
    const int64_t Tmax = aec_num_frames(nmax);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    AEC_ON_DEVICE(h);
    const bool nlms_batch = h->cfg.nlms_taps > 0 && !(B <= h->small_b && h->nlms_mode == 0);
    if (nlms_batch && nlms_smem_bytes(h->sched_len, h->cfg.nlms_taps) > 160 * 1024)   // before any launch
        return fail(h, AEC_ERR_UNSUPPORTED, "erb schedule too long for the NLMS kernel's LDS budget");
    const int nsig = near ? 3 : 2;
    // aec_process_prepared: the look-ahead pass named by `token` (aec_prepare_siglens), checked
    // before anything is launched; the pending ones queued before it are dropped (their slots stay
    // fenced by their done / freed events)
    aec_handle::PreSlot* ps = nullptr;
    if (token) {
        int k = 0;
        while (k < h->pre_count && h->pre[(h->pre_head + k) & 1].token != token) ++k;
        if (k == h->pre_count) return fail(h, AEC_ERR_INVALID_ARG, "look-ahead token not pending");
        aec_handle::PreSlot& c = h->pre[(h->pre_head + k) & 1];
        if (!(c.sig[0] == mic && c.sig[1] == ref && c.sig[2] == near && c.ld == ld && c.nsig == nsig &&
              c.l3.size() == (size_t)B * 3 &&
              std::memcmp(c.l3.data(), lengths3, (size_t)B * 3 * sizeof(int64_t)) == 0))
            return fail(h, AEC_ERR_INVALID_ARG, "look-ahead prepared for other signals / ld / B / lengths");
        ps = &c;
        h->pre_head = (h->pre_head + k + 1) & 1;
        h->pre_count -= k + 1;
        c.token = 0;
    }
    // a consumer of an earlier pipelined launch gave up waiting for its producer: that call's
    // output is invalid; reported once, here
    if (h->h_pipe_err && *reinterpret_cast<volatile int*>(h->h_pipe_err)) {
        *h->h_pipe_err = 0;
        return fail(h, AEC_ERR_HIP, "an earlier small-batch pipelined call timed out waiting for its producer blocks");
    }
    // this call overwrites the features a pending aec_train_backward would read
    h->train_B = 0;
    ++h->train_gen;
    aec_status s = begin_call(h, st);
    if (s != AEC_OK) return s;
    CallGuard cg{h, st};
    s = ensure_ws(h, B, Tmax);
    if (s != AEC_OK) return s;
    s = prepare_lists(h, lengths3, B, nsig_in, st);
    if (s != AEC_OK) return s;
    // the consumed slot is free again once this call's kernels have read its cvals (every exit)
    struct PreRelease {
        aec_handle::PreSlot* ps;
        hipStream_t st;
        ~PreRelease() {
            if (ps && hipEventRecord(ps->freed, st) == hipSuccess) ps->freed_rec = true;
        }
    } pre_rel{ps, st};
    const float* cvals = ps ? ps->cvals : h->d_cvals;
    // the pipelined split path: one GRU + synthesis launch of 2 B blocks (producers first) runs the
    // recursion and mic_erb too; it needs one block per CU for each and the one tap count it is
    // built for, and runs the GRU one stream per block (the AEC_GRU_NS rule for small batches)
    const bool pipe = h->small_pipe && h->cfg.nlms_taps == kPipeTaps && B <= h->small_b && h->nlms_mode == 0 &&
                      h->fused && h->gru_mode == 0 && 2 * (int64_t)B <= (int64_t)h->num_cus &&
                      AEC_MODE_KNOB("AEC_GRU_NS", 0) != 2;
    if (pipe) {
        if (B > h->progress_cap) {
            if (h->have_last) HIP_TRY(h, hipEventSynchronize(h->ev_last));
            if (h->d_progress) HIP_TRY(h, hipFree(h->d_progress));
            h->d_progress = nullptr;
            h->progress_cap = 0;
            HIP_TRY(h, hipMalloc(&h->d_progress, (size_t)B * sizeof(unsigned long long)));
            HIP_TRY(h, hipMemset(h->d_progress, 0, (size_t)B * sizeof(unsigned long long)));
            h->progress_cap = B;
        }
        if (!h->h_pipe_err) {
            HIP_TRY(h, hipHostMalloc(reinterpret_cast<void**>(&h->h_pipe_err), sizeof(int), hipHostMallocMapped));
            *h->h_pipe_err = 0;
            HIP_TRY(h, hipHostGetDevicePointer(reinterpret_cast<void**>(&h->d_pipe_err), h->h_pipe_err, 0));
        }
    }
    if (ps) HIP_TRY(h, hipStreamWaitEvent(st, ps->done, 0));
    mark(h, st);
    // the NLMS split path's K2 takes the normaliser scalars straight from the moment partials (the
    // same expression as norm_finalize_kernel): one launch fewer on the latency-bound small batches
    const bool split = h->cfg.nlms_taps > 0 && B <= h->small_b && h->nlms_mode == 0;
    // the bypass path (no NLMS) with up to half the CUs of streams: GRU + synthesis fused (one stream
    // per block) over K2's mic rows instead of gru_kernel + synthesis_kernel re-deriving the mic
    // spectrum (the same values, tested bit-exact)
    const bool bypass_fused = h->cfg.nlms_taps == 0 && h->fused && h->gru_mode == 0 &&
                              2 * (int64_t)B <= (int64_t)h->num_cus;
    const bool fold_norm = (split || bypass_fused) && !ps;
    if (!ps) {
        HIP_TRY(h, launch_moments(mic, ref, near, ld, h->d_slen, h->d_mom, 0, B, nsig, st));
        if (!fold_norm) HIP_TRY(h, launch_norm_finalize(h->d_mom, h->d_slen, h->d_cvals, 0, B, nsig, st));
    }
    if (split || bypass_fused) {
        // packed mic / ref rows of K2
        const size_t need = (size_t)B * Tmax * 512 + (size_t)B * 256;      // + one dummy row per stream
        if (need > h->rows_cap) {
            if (h->have_last) HIP_TRY(h, hipEventSynchronize(h->ev_last));
            if (h->d_rows) HIP_TRY(h, hipFree(h->d_rows));
            h->d_rows = nullptr;
            h->rows_cap = 0;
            HIP_TRY(h, hipMalloc(&h->d_rows, need * sizeof(float2)));
            h->rows_cap = need;
        }
    }
    if (split) {
        // few streams: transforms frame-parallel (K2 + rows), recursion per stream, mic_erb frame-parallel
        AnalysisArgs a{};
        a.sig[0] = mic; a.sig[1] = ref; a.sig[2] = near;
        a.ld = ld; a.items = h->d_items; a.nitems = h->nitems;
        a.num_cus = h->num_cus; a.cvals = fold_norm ? nullptr : cvals; a.mom = h->d_mom; a.slen = h->d_slen;
        a.tables = reinterpret_cast<const float*>(h->d_tab);
        a.sched = h->d_sched; a.sched_len = h->sched_len; a.nsig = nsig;
        a.feats = h->d_feats; a.Tmax = Tmax; a.rows = h->d_rows;
        mark(h, st);
        HIP_TRY(h, launch_analysis(a, st));
        if (!pipe) {
            HIP_TRY(h, launch_nlms_recursion(h->d_rows, h->d_spec, h->d_len, Tmax, h->cfg.nlms_taps, h->cfg.nlms_mu,
                                             h->cfg.nlms_beta, h->cfg.nlms_delta, 0, B,
                                             h->d_rows + (size_t)B * Tmax * 512, st));
            HIP_TRY(h, launch_mic_erb(h->d_spec, h->d_feats, h->d_len, Tmax, h->d_sched, h->sched_len, h->d_items,
                                      h->nitems, st));
        }
    } else if (h->cfg.nlms_taps > 0) {
        NlmsArgs a{};
        a.sig[0] = mic; a.sig[1] = ref; a.sig[2] = near;
        a.ld = ld; a.lens = h->d_len; a.slen = h->d_slen; a.b0 = 0; a.cvals = cvals;
        a.tables = reinterpret_cast<const float*>(h->d_tab);
        a.sched = h->d_sched; a.sched_len = h->sched_len; a.nsig = nsig;
        a.feats = h->d_feats; a.Tmax = Tmax; a.spec = h->d_spec;
        a.taps = h->cfg.nlms_taps; a.mu = h->cfg.nlms_mu; a.beta = h->cfg.nlms_beta; a.delta = h->cfg.nlms_delta;
        a.mode = h->nlms_mode;
        a.prio = h->nlms_prio;
        a.erb_role = h->nlms_erb;
        mark(h, st);
        HIP_TRY(h, launch_nlms_analysis(a, B, st));
    } else {
        AnalysisArgs a{};
        a.sig[0] = mic; a.sig[1] = ref; a.sig[2] = near;
        a.ld = ld; a.items = h->d_items; a.nitems = h->nitems;
        a.num_cus = h->num_cus; a.cvals = fold_norm ? nullptr : cvals; a.mom = h->d_mom; a.slen = h->d_slen;
        a.tables = reinterpret_cast<const float*>(h->d_tab);
        a.sched = h->d_sched; a.sched_len = h->sched_len; a.nsig = nsig;
        a.feats = h->d_feats; a.Tmax = Tmax;
        if (bypass_fused) a.rows = h->d_rows;
        mark(h, st);
        HIP_TRY(h, launch_analysis(a, st));
    }
    mark(h, st);

    GruArgs g{};
    g.feats = h->d_feats; g.Tmax = Tmax; g.lens = h->d_len; g.w = h->d_w;
    g.est = h->d_est; g.loss = loss; g.has_near = near != nullptr;
    g.dbg_h = h->debug ? h->d_dbg : nullptr;
    g.dbg_mask = h->debug ? h->d_dbg + B * Tmax * 32 : nullptr;
    g.mode = h->gru_mode;
    g.b0 = 0;

    SynthArgs y{};
    y.mic = mic; y.ld = ld; y.items = h->d_sitems; y.nitems = h->nsitems; y.num_cus = h->num_cus;
    y.cvals = cvals;
    y.tables = reinterpret_cast<const float*>(h->d_tab);
    y.bintab = h->d_bintab; y.est = h->d_est; y.Tmax = Tmax;
    y.out = out; y.ld_out = ld_out;
    y.spec = h->cfg.nlms_taps > 0 ? h->d_spec : (bypass_fused ? h->d_rows : nullptr);
    y.spec_stride = bypass_fused ? 512 : 256;
    y.fmode = h->fused_mode;
    if (pipe) {
        PipeArgs q{};
        q.rows = h->d_rows; q.spec = h->d_spec; q.feats = h->d_feats;
        q.sched = h->d_sched; q.sched_len = h->sched_len;
        q.mu = h->cfg.nlms_mu; q.beta = h->cfg.nlms_beta; q.delta = h->cfg.nlms_delta;
        q.progress = h->d_progress; q.epoch = ++h->pipe_epoch; q.err = h->d_pipe_err;
        q.spin_limit = 1 << 20;       // ~1-2 s of polls: far beyond any producer's lead
        // test hook: producers publish nothing and consumers give up after N polls (the timeout path:
        // this call's output is invalid, the handle's next call fails)
        const int stall = AEC_MODE_KNOB("AEC_SMALLB_PIPE_STALL", 0);
        if (stall > 0) {
            q.stall = 1;
            q.spin_limit = stall;
        }
        HIP_TRY(h, launch_gru_synth_pipe(g, y, q, B, st));
        mark(h, st);
        mark(h, st);
    } else if (y.spec && h->fused && h->gru_mode == 0) {
        // one kernel: the synthesis runs two chunks behind the recurrence
        HIP_TRY(h, launch_gru_synth(g, y, B, st));
        mark(h, st);
        mark(h, st);
    } else {
        HIP_TRY(h, launch_gru(g, B, st));
        mark(h, st);
        HIP_TRY(h, launch_synthesis(y, st));
        mark(h, st);
    }
    h->last_B = B;
    h->last_T = Tmax;
    return cg.end();
}

aec_status aec_prepare_siglens(aec_handle* h, const float* mic, const float* ref, const float* near,
                               const int64_t* lengths3, int32_t B, int64_t ld, void* stream, uint64_t* token) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (token) *token = 0;
    if (B <= 0 || !lengths3 || !mic || !ref) return fail(h, AEC_ERR_INVALID_ARG, "bad batch / lengths / signals");
    if (h->pre_count >= 2) return fail(h, AEC_ERR_INVALID_ARG, "two look-ahead batches already pending");
    const int nsig = near ? 3 : 2;
    for (int b = 0; b < B; ++b) {
        const int64_t n = lengths3[3 * b];
        for (int sg = 0; sg < nsig; ++sg) {
            const int64_t ns = lengths3[3 * b + sg];
            if (ns < 1 || ns > ld) return fail(h, AEC_ERR_INVALID_ARG, "length out of [1, ld]");
            if (ns > INT32_MAX - 4096) return fail(h, AEC_ERR_UNSUPPORTED, "stream longer than 2^31 - 4096 samples");
            if (ns / 256 != n / 256)
                return fail(h, AEC_ERR_INVALID_ARG, "ref / near frame count differs from mic's (N//256 + 1)");
        }
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    AEC_ON_DEVICE(h);
    aec_handle::PreSlot& ps = h->pre[(h->pre_head + h->pre_count) & 1];
    if (ps.used) HIP_TRY(h, hipEventSynchronize(ps.done));      // its staging copy has been read
    if (B > ps.cap) {
        if (ps.freed_rec) HIP_TRY(h, hipEventSynchronize(ps.freed));
        (void)hipFree(ps.mom); (void)hipFree(ps.cvals); (void)hipFree(ps.slen);
        if (ps.host) (void)hipHostFree(ps.host);
        ps.mom = nullptr; ps.cvals = nullptr; ps.slen = nullptr; ps.host = nullptr; ps.cap = 0;
        const int64_t cap = B + B / 4;
        HIP_TRY(h, hipMalloc(&ps.mom, (size_t)cap * 3 * kMomChunks * sizeof(double2)));
        HIP_TRY(h, hipMalloc(&ps.cvals, (size_t)cap * 3 * sizeof(float)));
        HIP_TRY(h, hipMalloc(&ps.slen, (size_t)cap * 4 * sizeof(int32_t)));
        HIP_TRY(h, hipHostMalloc(reinterpret_cast<void**>(&ps.host), (size_t)cap * 4 * sizeof(int32_t)));
        ps.cap = cap;
    }
    if (!ps.done) HIP_TRY(h, hipEventCreateWithFlags(&ps.done, hipEventDisableTiming));
    if (!ps.freed) HIP_TRY(h, hipEventCreateWithFlags(&ps.freed, hipEventDisableTiming));
    // the call that consumed this slot last has read its cvals; a dropped pass into it has finished
    if (ps.freed_rec) HIP_TRY(h, hipStreamWaitEvent(st, ps.freed, 0));
    if (ps.used) HIP_TRY(h, hipStreamWaitEvent(st, ps.done, 0));
    for (int b = 0; b < B; ++b) {   // prepare_lists' per-signal lengths
        for (int sg = 0; sg < 3; ++sg)
            ps.host[4 * b + sg] = (int32_t)(sg < nsig ? lengths3[3 * b + sg] : lengths3[3 * b]);
        ps.host[4 * b + 3] = 0;
    }
    HIP_TRY(h, hipMemcpyAsync(ps.slen, ps.host, (size_t)B * 4 * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(h, launch_moments(mic, ref, near, ld, ps.slen, ps.mom, 0, B, nsig, st));
    HIP_TRY(h, launch_norm_finalize(ps.mom, ps.slen, ps.cvals, 0, B, nsig, st));
    HIP_TRY(h, hipEventRecord(ps.done, st));
    ps.used = true;
    ps.sig[0] = mic; ps.sig[1] = ref; ps.sig[2] = near;
    ps.ld = ld;
    ps.nsig = nsig;
    ps.l3.assign(lengths3, lengths3 + (size_t)B * 3);
    ps.token = h->next_token++;
    if (token) *token = ps.token;
    ++h->pre_count;
    return AEC_OK;
}

aec_status aec_prepare(aec_handle* h, const float* mic, const float* ref, const float* near,
                       const int64_t* lengths, int32_t B, int64_t ld, void* stream, uint64_t* token) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (B <= 0 || !lengths) return fail(h, AEC_ERR_INVALID_ARG, "bad batch / lengths");
    std::vector<int64_t> l3((size_t)B * 3);
    for (int b = 0; b < B; ++b) l3[3 * b] = l3[3 * b + 1] = l3[3 * b + 2] = lengths[b];
    return aec_prepare_siglens(h, mic, ref, near, l3.data(), B, ld, stream, token);
}

aec_status aec_debug_copy(aec_handle* h, int32_t what, float* dst, size_t n, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    const int64_t B = h->last_B, T = h->last_T;
    if (!dst || n < (size_t)(B * T * 32)) return fail(h, AEC_ERR_INVALID_ARG, "dst too small");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    AEC_ON_DEVICE(h);
    if (what < 0 || what > 5) return fail(h, AEC_ERR_INVALID_ARG, "unknown intermediate");
    if ((what == 3 || what == 4) && !h->debug) return fail(h, AEC_ERR_INVALID_ARG, "enable aec_set_debug before aec_process");
    // ordered after the last call (it may have run on another stream) like any other call
    aec_status s = begin_call(h, st);
    if (s != AEC_OK) return s;
    CallGuard cg{h, st};
    if (what >= 0 && what <= 2) {
        HIP_TRY(h, hipMemcpy2DAsync(dst, 32 * sizeof(float), h->d_feats + 32 * what, 96 * sizeof(float),
                                    32 * sizeof(float), B * T, hipMemcpyDeviceToDevice, st));
    } else if (what == 3 || what == 4) {
        if (!h->debug) return fail(h, AEC_ERR_INVALID_ARG, "enable aec_set_debug before aec_process");
        HIP_TRY(h, hipMemcpyAsync(dst, h->d_dbg + (what - 3) * B * T * 32, B * T * 32 * sizeof(float),
                                  hipMemcpyDeviceToDevice, st));
    } else {
        HIP_TRY(h, hipMemcpyAsync(dst, h->d_est, B * T * 32 * sizeof(float), hipMemcpyDeviceToDevice, st));
    }
    return cg.end();
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

aec_status aec_erb_tables_check(const float* erb, const float* mags, const float* est, float* bands,
                                float* gains, int32_t* sched_len, int32_t* conflicts) {
    if (!erb || !mags || !est || !bands || !gains) return AEC_ERR_INVALID_ARG;
    const ErbTables t = build_erb_tables(erb);
    if (!t.ok) return AEC_ERR_UNSUPPORTED;
    const int L = t.sched_len;
    float part[48];
    for (int l = 0; l < 16; ++l) {
        float a[3] = {0.f, 0.f, 0.f};
        for (int e = 0; e < L; ++e) {
            const float* en = &t.sched[((size_t)e * 16 + l) * 4];
            int k;
            std::memcpy(&k, en, 4);
            for (int s = 0; s < 3; ++s) a[s] = std::fma(en[1 + s], mags[k], a[s]);
        }
        for (int s = 0; s < 3; ++s) part[3 * l + s] = a[s];
    }
    int comb[64];
    std::memcpy(comb, &t.sched[(size_t)L * 16 * 4], sizeof(comb));
    for (int j = 0; j < 32; ++j) bands[j] = part[comb[2 * j]] + (comb[2 * j + 1] >= 0 ? part[comb[2 * j + 1]] : 0.f);
    for (int k = 0; k < 257; ++k) {
        const float* e = &t.bintab[k * 4];
        int ja, jb;
        std::memcpy(&ja, &e[0], 4);
        std::memcpy(&jb, &e[2], 4);
        gains[k] = e[1] * est[ja] + e[3] * est[jb];
    }
    if (sched_len) *sched_len = L;
    if (conflicts) *conflicts = t.conflicts;
    return AEC_OK;
}

aec_status aec_stream_open(aec_handle* h, int32_t B) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (B < 1) return fail(h, AEC_ERR_INVALID_ARG, "stream count must be >= 1");
    AEC_ON_DEVICE(h);
    HIP_TRY(h, hipDeviceSynchronize());   // a previous state may still be in use
    if (h->d_state) { HIP_TRY(h, hipFree(h->d_state)); h->d_state = nullptr; }
    h->stream_B = 0;
    const int64_t stride = stream_state_floats(h->cfg.nlms_taps);
    HIP_TRY(h, hipMalloc(&h->d_state, (size_t)B * stride * sizeof(float)));
    HIP_TRY(h, hipMemset(h->d_state, 0, (size_t)B * stride * sizeof(float)));
    h->stream_B = B;
    h->stream_stride = stride;
    return AEC_OK;
}

aec_status aec_stream_reset(aec_handle* h, int32_t b, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!h->d_state) return fail(h, AEC_ERR_INVALID_ARG, "aec_stream_open first");
    if (b < -1 || b >= h->stream_B) return fail(h, AEC_ERR_INVALID_ARG, "stream index out of range");
    AEC_ON_DEVICE(h);
    const int64_t first = b < 0 ? 0 : b, count = b < 0 ? h->stream_B : 1;
    HIP_TRY(h, hipMemsetAsync(h->d_state + first * h->stream_stride, 0, (size_t)count * h->stream_stride * sizeof(float),
                              reinterpret_cast<hipStream_t>(stream)));
    return AEC_OK;
}

aec_status aec_stream_step(aec_handle* h, const float* mic, const float* ref, int64_t ld_in, float* out,
                           int64_t ld_out, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!h->d_state) return fail(h, AEC_ERR_INVALID_ARG, "aec_stream_open first");
    if (!h->have_w || !h->have_erb) return fail(h, AEC_ERR_INVALID_ARG, "weights / erb not set");
    if (!mic || !ref || !out) return fail(h, AEC_ERR_INVALID_ARG, "null mic / ref / out");
    if (ld_in < 256 || ld_out < 256) return fail(h, AEC_ERR_INVALID_ARG, "ld_in / ld_out must be >= 256");
    AEC_ON_DEVICE(h);
    StreamStepArgs a{};
    a.mic = mic; a.ref = ref; a.ld_in = ld_in; a.out = out; a.ld_out = ld_out;
    a.state = h->d_state; a.state_stride = h->stream_stride;
    a.w = h->d_w; a.tables = reinterpret_cast<const float*>(h->d_tab);
    a.sched = h->d_sched; a.sched_len = h->sched_len; a.bintab = h->d_bintab;
    a.mu = h->cfg.nlms_mu; a.beta = h->cfg.nlms_beta; a.delta = h->cfg.nlms_delta;
    HIP_TRY(h, launch_stream_step(a, h->stream_B, h->cfg.nlms_taps, reinterpret_cast<hipStream_t>(stream)));
    return AEC_OK;
}

// ---------------------------------------------------------------------------
// Training step (scripts/train1.py:191-218; kernels in aec_train.hip)
// ---------------------------------------------------------------------------
aec_status aec_set_weights_device(aec_handle* h, const float* w, size_t n, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!w || n != kWeights32) return fail(h, AEC_ERR_INVALID_ARG, "weights blob must hold 12544 floats");
    AEC_ON_DEVICE(h);
    // stream-ordered after the handle's last call (on whichever stream it ran), which may still
    // read the old blob; kernels of this call's stream that follow see the new one
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    aec_status s = begin_call(h, st);
    if (s != AEC_OK) return s;
    CallGuard cg{h, st};
    HIP_TRY(h, hipMemcpyAsync(h->d_w, w, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    h->have_w = true;
    return cg.end();
}

aec_status aec_train_forward(aec_handle* h, const float* mic, const float* ref, const float* near, int64_t n,
                             int32_t B, int64_t ld, float* out, int64_t ld_out, float* loss, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!h->have_w || !h->have_erb) return fail(h, AEC_ERR_INVALID_ARG, "weights / erb not set");
    if (h->cfg.nlms_taps != 0)
        return fail(h, AEC_ERR_UNSUPPORTED, "training is the reference network's (nlms_taps = 0)");
    if (B < 1 || n < 1 || n > ld) return fail(h, AEC_ERR_INVALID_ARG, "need B >= 1 and 1 <= n <= ld");
    if (n > INT32_MAX - 4096) return fail(h, AEC_ERR_UNSUPPORTED, "stream longer than 2^31 - 4096 samples");
    if (!mic || !ref || !near || !loss) return fail(h, AEC_ERR_INVALID_ARG, "mic, ref, near and loss are required");
    if (out && aec_out_len(n) > ld_out) return fail(h, AEC_ERR_INVALID_ARG, "ld_out too small");
    const int64_t T = aec_num_frames(n);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    AEC_ON_DEVICE(h);
    aec_status s = begin_call(h, st);
    if (s != AEC_OK) return s;
    CallGuard cg{h, st};
    s = ensure_ws(h, B, T);
    if (s != AEC_OK) return s;
    const int64_t frames = (int64_t)B * T;
    const int nblk = train_wgrad_blocks(B, (int)T, h->num_cus);
    if (frames > h->train_cap || B > h->train_rows || nblk > h->part_cap) {
        HIP_TRY(h, hipDeviceSynchronize());
        (void)hipFree(h->d_th); (void)hipFree(h->d_tloss); (void)hipFree(h->d_rec); (void)hipFree(h->d_dg);
        (void)hipFree(h->d_part);
        h->d_th = h->d_tloss = h->d_rec = h->d_dg = h->d_part = nullptr;
        h->train_cap = 0; h->train_rows = 0; h->part_cap = 0;
        const int64_t fc = std::max(frames, h->ws_B * h->ws_T);
        HIP_TRY(h, hipMalloc(&h->d_th, (size_t)h->ws_B * h->ws_T * 32 * sizeof(float)));
        HIP_TRY(h, hipMalloc(&h->d_tloss, (size_t)h->ws_B * sizeof(float)));
        HIP_TRY(h, hipMalloc(&h->d_rec, (size_t)fc * 256 * sizeof(float)));
        HIP_TRY(h, hipMalloc(&h->d_dg, (size_t)fc * 128 * sizeof(float)));
        const int pc = std::max(nblk, 2 * h->num_cus);
        HIP_TRY(h, hipMalloc(&h->d_part, (size_t)pc * kWeights * sizeof(float)));
        h->train_cap = fc; h->train_rows = (int32_t)h->ws_B; h->part_cap = pc;
    }
    // collate_fn (train1.py:43-74) pads every row to n: one length for all
    std::vector<int64_t> l3((size_t)B * 3, n);
    s = prepare_lists(h, l3.data(), B, 3, st);
    if (s != AEC_OK) return s;
    const int64_t Tmax = T;
    HIP_TRY(h, launch_moments(mic, ref, near, ld, h->d_slen, h->d_mom, 0, B, 3, st));
    HIP_TRY(h, launch_norm_global(h->d_mom, B, n, h->d_cvals, st));
    AnalysisArgs a{};
    a.sig[0] = mic; a.sig[1] = ref; a.sig[2] = near;
    a.ld = ld; a.items = h->d_items; a.nitems = h->item_off[B];
    a.num_cus = h->num_cus; a.cvals = h->d_cvals; a.slen = h->d_slen;
    a.tables = reinterpret_cast<const float*>(h->d_tab);
    a.sched = h->d_sched; a.sched_len = h->sched_len; a.nsig = 3;
    a.feats = h->d_feats; a.Tmax = Tmax;
    HIP_TRY(h, launch_analysis(a, st));
    GruArgs g{};
    g.feats = h->d_feats; g.Tmax = Tmax; g.lens = h->d_len; g.w = h->d_w;
    g.est = h->d_est; g.loss = h->d_tloss; g.has_near = 1;
    g.dbg_h = h->d_th;
    g.mode = 0;
    g.b0 = 0;
    HIP_TRY(h, launch_gru(g, B, st));
    if (out) {
        SynthArgs y{};
        y.mic = mic; y.ld = ld; y.items = h->d_sitems; y.nitems = h->sitem_off[B]; y.num_cus = h->num_cus;
        y.cvals = h->d_cvals;
        y.tables = reinterpret_cast<const float*>(h->d_tab);
        y.bintab = h->d_bintab; y.est = h->d_est; y.Tmax = Tmax;
        y.out = out; y.ld_out = ld_out;
        HIP_TRY(h, launch_synthesis(y, st));
    }
    HIP_TRY(h, launch_loss_sum(h->d_tloss, B, loss, st));
    h->last_B = B;
    h->last_T = Tmax;
    h->train_B = B;
    h->train_T = (int32_t)T;
    ++h->train_gen;
    return cg.end();
}

int64_t aec_train_generation(const aec_handle* h) { return h ? h->train_gen : -1; }

aec_status aec_train_backward(aec_handle* h, const float* grad_loss, float* grad, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (h->train_B < 1) return fail(h, AEC_ERR_INVALID_ARG, "aec_train_backward before aec_train_forward");
    if (!grad) return fail(h, AEC_ERR_INVALID_ARG, "null grad");
    AEC_ON_DEVICE(h);
    TrainArgs t{};
    t.feats = h->d_feats; t.h = h->d_th; t.w = h->d_w;
    t.rec = h->d_rec; t.dg = h->d_dg; t.part = h->d_part;
    t.B = h->train_B; t.T = h->train_T; t.Tmax = h->train_T; t.num_cus = h->num_cus;
    const int nblk = train_wgrad_blocks(t.B, t.T, h->num_cus);
    if (nblk > h->part_cap) return fail(h, AEC_ERR_INVALID_ARG, "training workspace changed since the forward");
    if (!h->bptt_serial) {
        const int64_t nc = train_scan_chunks(t.T);
        const int64_t need = (int64_t)t.B * nc * (1024 + 64);
        if (need > h->scan_cap) {
            HIP_TRY(h, hipDeviceSynchronize());
            (void)hipFree(h->d_scan);
            h->d_scan = nullptr;
            h->scan_cap = 0;
            HIP_TRY(h, hipMalloc(&h->d_scan, (size_t)need * sizeof(float)));
            h->scan_cap = need;
        }
        t.scan_p = h->d_scan;
        t.scan_q = h->d_scan + (size_t)t.B * nc * 1024;
        t.scan_g = t.scan_q + (size_t)t.B * nc * 32;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    aec_status s = begin_call(h, st);
    if (s != AEC_OK) return s;
    CallGuard cg{h, st};
    HIP_TRY(h, launch_train_backward(t, nblk, grad_loss, grad, st));
    return cg.end();
}

aec_status aec_adam_step(aec_handle* h, float* params, const float* grad, float* exp_avg, float* exp_avg_sq,
                         size_t n, int64_t step, float lr, float beta1, float beta2, float eps, float weight_decay,
                         void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (!params || !grad || !exp_avg || !exp_avg_sq) return fail(h, AEC_ERR_INVALID_ARG, "null buffer");
    if (step < 1) return fail(h, AEC_ERR_INVALID_ARG, "step counts from 1");
    if (!(lr >= 0.f) || !(beta1 >= 0.f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f) || !(eps >= 0.f) ||
        !(weight_decay >= 0.f))
        return fail(h, AEC_ERR_INVALID_ARG, "Adam hyper-parameters out of range");
    AEC_ON_DEVICE(h);
    // torch/optim/adam.py computes the bias corrections in double on the host
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    HIP_TRY(h, launch_adam(params, grad, exp_avg, exp_avg_sq, (int64_t)n, beta1, beta2, eps, weight_decay,
                           (float)(lr / bc1), (float)std::sqrt(bc2), reinterpret_cast<hipStream_t>(stream)));
    return AEC_OK;
}

aec_status aec_adam_step_multi(aec_handle* h, float* const* params, const float* const* grads, float* const* exp_avg,
                               float* const* exp_avg_sq, const int64_t* sizes, const int64_t* steps, int32_t count,
                               float lr, float beta1, float beta2, float eps, float weight_decay, void* stream) {
    if (!h) return AEC_ERR_INVALID_ARG;
    if (count < 0 || (count > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !sizes || !steps)))
        return fail(h, AEC_ERR_INVALID_ARG, "null tensor list");
    if (!(lr >= 0.f) || !(beta1 >= 0.f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f) || !(eps >= 0.f) ||
        !(weight_decay >= 0.f))
        return fail(h, AEC_ERR_INVALID_ARG, "Adam hyper-parameters out of range");
    AEC_ON_DEVICE(h);
    for (int32_t c0 = 0; c0 < count; c0 += kAdamMax) {
        AdamList L{};
        L.n = std::min<int32_t>(kAdamMax, count - c0);
        L.off[0] = 0;
        for (int k = 0; k < L.n; ++k) {
            const int i = c0 + k;
            if (!params[i] || !grads[i] || !exp_avg[i] || !exp_avg_sq[i] || sizes[i] < 0 || steps[i] < 1)
                return fail(h, AEC_ERR_INVALID_ARG, "bad tensor in the list");
            L.p[k] = params[i]; L.g[k] = grads[i]; L.m[k] = exp_avg[i]; L.v[k] = exp_avg_sq[i];
            const double bc1 = 1.0 - std::pow((double)beta1, (double)steps[i]);
            const double bc2 = 1.0 - std::pow((double)beta2, (double)steps[i]);
            L.step_size[k] = (float)(lr / bc1);
            L.bc2_sqrt[k] = (float)std::sqrt(bc2);
            L.off[k + 1] = L.off[k] + sizes[i];
        }
        HIP_TRY(h, launch_adam_multi(L, beta1, beta2, eps, weight_decay, reinterpret_cast<hipStream_t>(stream)));
    }
    return AEC_OK;
}

void aec_destroy(aec_handle* h) {
    if (!h) return;
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    DeviceGuard dg(h->device);
    if (h->have_last) (void)hipEventSynchronize(h->ev_last);
    if (h->ev_last) (void)hipEventDestroy(h->ev_last);
    for (auto& sl : h->slots) {
        if (sl.pending) (void)hipEventSynchronize(sl.ev);
        if (sl.ev) (void)hipEventDestroy(sl.ev);
        if (sl.host) (void)hipHostFree(sl.host);
    }
    (void)hipFree(h->d_w); (void)hipFree(h->d_tab); (void)hipFree(h->d_sched); (void)hipFree(h->d_bintab);
    for (auto& ps : h->pre) {
        if (ps.used) (void)hipEventSynchronize(ps.done);
        if (ps.freed_rec) (void)hipEventSynchronize(ps.freed);
        (void)hipFree(ps.mom); (void)hipFree(ps.cvals); (void)hipFree(ps.slen);
        if (ps.host) (void)hipHostFree(ps.host);
        if (ps.done) (void)hipEventDestroy(ps.done);
        if (ps.freed) (void)hipEventDestroy(ps.freed);
    }
    (void)hipFree(h->d_mom); (void)hipFree(h->d_cvals); (void)hipFree(h->d_lists);
    (void)hipFree(h->d_feats); (void)hipFree(h->d_est); (void)hipFree(h->d_dbg); (void)hipFree(h->d_spec);
    (void)hipFree(h->d_state); (void)hipFree(h->d_rows); (void)hipFree(h->d_progress);
    if (h->h_pipe_err) (void)hipHostFree(h->h_pipe_err);
    (void)hipFree(h->d_th); (void)hipFree(h->d_tloss); (void)hipFree(h->d_rec); (void)hipFree(h->d_dg);
    (void)hipFree(h->d_part); (void)hipFree(h->d_scan);
    delete h;
}

}  // extern "C"
