// Native executor of one U2GNN encoder layer (torch TransformerEncoderLayer(d, nhead=1, ff,
// dropout), post-LN, slot-0 rows) — forward and backward issued from C++ straight onto HIP
// streams, one C-ABI call per layer instead of ~40 Python-side launches.
//
// Reference: pytorch_U2GNN_Sup.py:19-21,35 (UnSup: pytorch_U2GNN_UnSup.py:37-40,57) reach this
// through torch.nn.TransformerEncoder; the Python orchestration of the same kernels is
// u2gnn_hip/engine.py (encoder_layer_forward / encoder_layer_backward), which this file mirrors
// launch for launch (same tiles, split counts and reduction order, hence bit-identical results:
// tests/test_native_layer_gpu.py).
//
// Memory: every buffer is caller-allocated.  The forward writes the tensors saved for the
// backward into a "ctx" arena and uses a scratch workspace for S and split-K slabs; the backward
// carves all of its temporaries from one workspace with a bump allocator that never reuses a
// byte within a call, so work left running on the side stream cannot be overwritten by the main
// stream.  Sizes come from the same code run in planning mode (no launches).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <algorithm>
#include <atomic>
#include <vector>

#include "u2gnn_hip.h"

namespace {

inline int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// padded rows: multiples of 256 from 1024 rows on (the N^2 products always get 256x128 blocks),
// else of 128 (mirrors engine.row_pad)
inline int64_t rows_pad(int64_t N) { return N >= 1024 ? rup(N, 256) : rup(N, 128); }

struct Dims {
    int64_t N, d, ff, Np, dp, ffp;
    int prec;
    int prec_ab;   // dS, dQ, dK products (U2GNN_LAYER_ATTN_BWD_BF16: plain bf16)
    int prec_fwd;  // forward products (U2GNN_LAYER_FWD_F32: exact fp32; U2GNN_LAYER_FWD_X6: bf16x6)
    bool deep_wgrad;
    int window;   // 0: attention over all N rows; W: within windows of W rows (N % W == 0)
};

Dims make_dims(const u2gnn_layer_dims *a) {
    Dims D;
    D.N = a->N;
    D.d = a->d;
    D.ff = a->ff;
    D.Np = rows_pad(a->N);
    D.dp = rup(a->d, 64);
    D.ffp = rup(a->ff, 64);
    D.prec = a->precision;
    D.prec_ab = (a->precision == U2GNN_PREC_BF16X3 && (a->flags & U2GNN_LAYER_ATTN_BWD_BF16)) ? U2GNN_PREC_BF16
                                                                                             : a->precision;
    D.prec_fwd = a->precision;
    if (a->precision == U2GNN_PREC_BF16X3 && (a->flags & U2GNN_LAYER_FWD_F32)) D.prec_fwd = U2GNN_PREC_F32;
    if (a->precision == U2GNN_PREC_BF16X3 && (a->flags & U2GNN_LAYER_FWD_X6)) D.prec_fwd = U2GNN_PREC_BF16X6;
    if (a->precision == U2GNN_PREC_BF16X3 && (a->flags & U2GNN_LAYER_FWD_H3)) D.prec_fwd = U2GNN_PREC_F16X3;
    D.deep_wgrad = (a->flags & U2GNN_LAYER_DEEP_WGRAD) != 0;
    D.window = a->window;
    return D;
}

// bump allocator over a caller buffer; plan mode (base == nullptr) only counts
struct Arena {
    char *base;
    int64_t used = 0, cap;
    bool overflow = false;
    Arena(void *b, int64_t c) : base(static_cast<char *>(b)), cap(c) {}
    template <typename T>
    T *take(int64_t n) {
        const int64_t bytes = rup(n * (int64_t)sizeof(T), 256);
        T *p = base ? reinterpret_cast<T *>(base + used) : nullptr;
        used += bytes;
        if (base && used > cap) overflow = true;
        return p;
    }
    bool plan() const { return base == nullptr; }
};

// U2GNN_DEBUG=1 in the environment names the failing call on stderr
bool debug_on() {
    static const int on = [] {
        const char *e = std::getenv("U2GNN_DEBUG");
        return e && e[0] == '1' ? 1 : 0;
    }();
    return on != 0;
}

#define U2GNN_TRY(x)                                                                                \
    do {                                                                                            \
        const int rc_ = (x);                                                                        \
        if (rc_ != U2GNN_OK) {                                                                      \
            if (debug_on()) std::fprintf(stderr, "u2gnn: %s:%d: %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
            return rc_;                                                                             \
        }                                                                                           \
    } while (0)

struct Ctx {   // tensors saved by the forward for the backward
    // Pd: with dropout the signed probability image (P/(1-p) where kept, -P where dropped), else P
    float *QKV, *Pd, *O, *Z1, *X1, *mean1, *rstd1, *Hd, *Z2, *mean2, *rstd2;
    float *Psave;   // window mode: [N/W, W, W] probabilities
    float *stats;   // small-width node attention (d <= 32): its context (row statistics + compact Q, K, V)
};

// node attention for d <= 32 on the vector ALUs (u2gnn_attn_small_*, small_layer.hip): every precision, no
// N x N image (engine.small_attn mirrors the rule)
bool small_attn(const Dims &D) { return !D.window && D.d <= 32; }
// the forward tail (a3.3 + a3.4) of a mid-width layer with few rows as one row-block kernel + the slab LayerNorm
// (mid_layer.hip; C2: 2 launches instead of 5); engine.mid_tail mirrors the rule
bool mid_tail(const Dims &D) { return !D.window && D.d > 32 && D.dp <= 256 && D.Np <= 512; }

Ctx carve_ctx(Arena &A, const Dims &D, bool drop) {
    Ctx c;
    // the small-width path projects straight into its compact attention context: no [Np][3 dp] image
    c.QKV = small_attn(D) ? nullptr : A.take<float>(D.Np * 3 * D.dp);
    (void)drop;
    c.Pd = c.Psave = c.stats = nullptr;
    if (D.window)
        c.Psave = A.take<float>(D.N * D.window);
    else if (small_attn(D))
        c.stats = A.take<float>(u2gnn_attn_small_ctx_floats(D.Np, D.d));
    else
        c.Pd = A.take<float>(D.Np * D.Np);
    c.O = A.take<float>(D.Np * D.dp);
    c.Z1 = A.take<float>(D.Np * D.dp);
    c.X1 = A.take<float>(D.Np * D.dp);
    c.mean1 = A.take<float>(D.Np);
    c.rstd1 = A.take<float>(D.Np);
    c.Hd = A.take<float>(D.Np * D.ffp);
    c.Z2 = A.take<float>(D.Np * D.dp);
    c.mean2 = A.take<float>(D.Np);
    c.rstd2 = A.take<float>(D.Np);
    return c;
}

// live launch timing of one role (u2gnn_probe_arm / u2gnn_probe_collect): a diagnostic of the bench, the one
// piece of process-wide state of the executor.  Every access holds g_probe_mu (arm, mark and collect may come
// from different host threads); an unarmed probe costs one relaxed atomic load per mark.
struct Probe {
    int role = 0, cap = 0, n = 0;
    hipEvent_t *ev = nullptr;   // [2 * cap]: start, end
};
Probe g_probe;
std::mutex g_probe_mu;
std::atomic<int> g_probe_role{0};

void probe_mark(int role, bool end, hipStream_t st, bool plan) {
    if (plan || g_probe_role.load(std::memory_order_relaxed) != role) return;
    std::lock_guard<std::mutex> lk(g_probe_mu);
    if (g_probe.role != role || g_probe.n >= g_probe.cap) return;
    (void)hipEventRecord(g_probe.ev[2 * g_probe.n + (end ? 1 : 0)], st);
    if (end) ++g_probe.n;
}

// f16x3 operand pre-scale exponents (u2gnn_hip.h h3_exp_a / h3_exp_b; kernels.H3_EXP / h3_prob_exp mirror them):
// activations and weights by 2^6, the probability image (entries ~1/N, at most 1/(1-p)) by 2^(15 - ceil(log2(1/(1-p))))
constexpr int32_t kH3Exp = 6;
int32_t h3_prob_exp(float pd) {
    int32_t e = 15;
    for (float m = 1.f / (1.f - pd); m > 1.f; m *= 0.5f) --e;
    return e;
}

struct G {   // one GEMM launch (defaults = plain store)
    u2gnn_gemm_args a;
    G(const float *A, const float *B, float *C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
      int64_t ldc, int prec) {
        std::memset(&a, 0, sizeof(a));
        a.A = A, a.B = B, a.C = C, a.M = M, a.N = N, a.K = K, a.lda = lda, a.ldb = ldb, a.ldc = ldc;
        a.epilogue = U2GNN_EPI_STORE;
        a.split_k = 1;
        a.alpha = 1.f;
        a.precision = prec;
        if (prec == U2GNN_PREC_F16X3) a.h3_exp_a = a.h3_exp_b = kH3Exp;
    }
    G &ta() { a.trans_a = 1; return *this; }
    G &tb() { a.trans_b = 1; return *this; }
    G &epi(int e) { a.epilogue = e; return *this; }
    G &tile(int t) { a.tile = t; return *this; }
    int run(hipStream_t st, bool plan) { return plan ? U2GNN_OK : u2gnn_gemm(&a, st); }
};

hipEvent_t pooled_event();

// Reductions (and weight-gradient products) held back to the end of a latency-bound layer's backward,
// where they go out as one grouped GEMM launch and one u2gnn_reduce_batch call (<= 2 launches) instead
// of 12-16 launches of a few microseconds each.  Used when the layer runs on one stream (no side stream:
// C5, C2, C3).  Every job computes the same bits as its immediate launch (u2gnn_hip.h, ABI v11).
struct Defer {
    std::vector<u2gnn_reduce_job> red;
    std::vector<u2gnn_gemm_args> gemm;
    std::vector<int> role;   // probe role of each held-back GEMM
    bool gemms = false;   // hold back the GEMM launches as well (one grouped launch)
};

int flush(Defer *df, Arena &W, hipStream_t st) {
    if (!df) return U2GNN_OK;
    const bool plan = W.plan();
    for (size_t o = 0; o < df->gemm.size(); o += 8) {
        const size_t n = std::min<size_t>(8, df->gemm.size() - o);
        // a grouped launch is timed as a whole under each role it carries (u2gnn_probe_arm)
        int probed = 0;
        for (size_t i = o; i < o + n; ++i)
            if (df->role[i] && df->role[i] != probed) probed = df->role[i], probe_mark(probed, false, st, plan);
        if (!plan) U2GNN_TRY(u2gnn_gemm_group(df->gemm.data() + o, (int32_t)n, st));
        probed = 0;
        for (size_t i = o; i < o + n; ++i)
            if (df->role[i] && df->role[i] != probed) probed = df->role[i], probe_mark(probed, true, st, plan);
    }
    const int64_t wsf = u2gnn_reduce_batch_ws_floats(df->red.data(), (int32_t)df->red.size());
    if (wsf < 0) return U2GNN_E_ARG;
    float *ws = W.take<float>(wsf > 0 ? wsf : 1);
    if (!plan && !df->red.empty())
        U2GNN_TRY(u2gnn_reduce_batch(df->red.data(), (int32_t)df->red.size(), ws, wsf, st));
    df->red.clear();
    df->gemm.clear();
    df->role.clear();
    return U2GNN_OK;
}

u2gnn_reduce_job rjob(int kind) {
    u2gnn_reduce_job j;
    std::memset(&j, 0, sizeof(j));
    j.kind = kind;
    j.alpha = 1.f;
    return j;
}

// split-K block targets (engine._gemm_split): 448 blocks for 64 / 128 tiles, 240 for 256x128 tiles
// (round-2 sweeps: 224 / 896 within noise, 120 / 300 / 460 slower on the 256x128 products)
constexpr int64_t kSplitTarget = 448, kSplitTarget256 = 240;

// engine._gemm_split: deterministic split-K into fp32 slabs + one reduce pass (alpha, accumulate,
// padded->real block map).  deep = weight gradient (16-deep K step, <= 8 slabs).  red_st: run the
// reduce pass on that stream after the GEMM (pooled fork event; the caller joins it back).
int gemm_split(Arena &W, const Dims &D, const float *A, const float *B, float *C, int64_t M, int64_t N, int64_t Kd,
               int64_t lda, int64_t ldb, int64_t ldc, bool ta, float alpha, bool accumulate, const int64_t *rblk,
               const int64_t *cblk, bool deep, hipStream_t st, bool clamp_a = false, int prec = -1, int role = 0,
               hipStream_t red_st = nullptr, Defer *df = nullptr, float **slabs_out = nullptr,
               int64_t *nslab_out = nullptr, int32_t h3_exp_a = kH3Exp) {
    if (prec < 0) prec = D.prec;
    const bool f32 = prec == U2GNN_PREC_F32;
    const int64_t bk = f32 ? 16 : 32;
    const bool plan = W.plan();
    const bool mapped = rblk != nullptr;
    // (tiny: an accumulating product of at most 16 tiles and 16 K steps -- C2's dX += dQKV W_in, 4 tiles --
    // runs as one short launch instead of 3 split-K blocks + a reduce launch; engine._gemm_split mirrors it)
    const bool tiny = accumulate && Kd <= 512 && (M / 64) * (N / 64) <= 16;
    if (!f32 && !deep && !mapped && Kd <= 2048 && M % 64 == 0 && N % 64 == 0 &&
        ((M / 64) * (N / 64) >= 256 || tiny)) {
        // shallow K (dH.W1, dQKV.W_in) with enough 64x64 tiles to fill the chip: no split, the
        // epilogue accumulates straight into C (no slabs, no reduce pass)
        G g(A, B, C, M, N, Kd, lda, ldb, ldc, prec);
        if (ta) g.ta();
        g.a.alpha = alpha;
        g.a.clamp_a = clamp_a;
        if (prec == U2GNN_PREC_F16X3) g.a.h3_exp_a = h3_exp_a;
        const bool big = M % 256 == 0 && N % 128 == 0 && (M / 256) * (N / 128) >= U2GNN_BIG_TILE_BLOCKS;
        g.epi(accumulate ? U2GNN_EPI_ACCUM : U2GNN_EPI_STORE).tile(big ? 256 : 64);
        probe_mark(role, false, st, plan);
        const int rc = g.run(st, plan);
        probe_mark(role, true, st, plan);
        return rc;
    }
    int t;
    int64_t tiles, target = kSplitTarget;
    if (!f32 && M % 256 == 0 && N % 128 == 0 && (M / 256) * (N / 128) >= 32) {
        t = 256, tiles = (M / 256) * (N / 128), target = kSplitTarget256;
        // dQ and dK go out as ONE grouped launch: half the block target each, so the launch holds ~240 blocks
        // (C4: split 2, 228 blocks instead of split 4 and 456; 3.016-3.017 vs 3.054-3.065 ms per step in one
        // session, profiles/r04/ab_sched.txt; split 1 and 128x128 tiles at split 2 were slower)
        if (role == U2GNN_ROLE_DQ || role == U2GNN_ROLE_DK) target = kSplitTarget256 / 2;
    } else {
        t = (M % 128 == 0 && N % 128 == 0) ? 128 : 64;
        tiles = (M / t) * (N / t);
    }
    int64_t split = target / (tiles > 0 ? tiles : 1);
    if (Kd / (4 * bk) < split) split = Kd / (4 * bk);
    if (split < 1) split = 1;
    // slab cap of the weight gradients (engine.wgrad_split_cap): 8 for node-sized depths, 16 for
    // token-sized ones (neighbour mode, K = N(k+1) rows)
    const int64_t wgrad_split_max = Kd <= 8192 ? 8 : 16;
    if (deep && D.deep_wgrad && !f32 && t == 128) {
        t = 129;
        split = target / (tiles > 0 ? tiles : 1);
        if (split > wgrad_split_max) split = wgrad_split_max;
        if (split < 1) split = 1;
    }
    // a held-back product joins its layer's grouped launch, whose kernels are the 64x64, 16-deep 128x128 and
    // 256x128 ones: a 128x128 job runs there as four 64x64 tiles (the split is chosen above, so the sums and
    // bits are the same; C2's dV, dQ, dK: one launch instead of three)
    // A launch of fewer than 64 blocks of 128x128 runs them as 64x64 tiles too (4x the blocks for the same
    // sums; C2's dX1 = dH W1: 8 blocks of a 4-step K loop, 8.6 us)
    // (bf16 precisions, whose 64x64 and 128x128 kernels form the same k-ordered sums)
    const int t_group = (!f32 && t == 128 && ((df && df->gemms) || (M / 128) * (N / 128) * split < 64)) ? 64 : t;
    if (split == 1 && !mapped) {
        G g(A, B, C, M, N, Kd, lda, ldb, ldc, prec);
        if (ta) g.ta();
        g.a.alpha = alpha;
        g.a.clamp_a = clamp_a;
        if (prec == U2GNN_PREC_F16X3) g.a.h3_exp_a = h3_exp_a;
        g.epi(accumulate ? U2GNN_EPI_ACCUM : U2GNN_EPI_STORE).tile(t_group);
        if (df && df->gemms && !accumulate) {
            df->gemm.push_back(g.a);
            df->role.push_back(role);
            return U2GNN_OK;
        }
        probe_mark(role, false, st, plan);
        const int rc = g.run(st, plan);
        probe_mark(role, true, st, plan);
        return rc;
    }
    float *slabs = W.take<float>(split * M * N);
    G g(A, B, slabs, M, N, Kd, lda, ldb, N, prec);
    if (ta) g.ta();
    g.a.split_k = (int32_t)split;
    g.a.slab_stride = M * N;
    g.a.clamp_a = clamp_a;
    if (prec == U2GNN_PREC_F16X3) g.a.h3_exp_a = h3_exp_a;
    g.tile(t_group);
    const int64_t rb0 = rblk ? rblk[0] : M, rb1 = rblk ? rblk[1] : M;
    const int64_t cb0 = cblk ? cblk[0] : N, cb1 = cblk ? cblk[1] : N;
    if (df) {   // slab reduce (and with df->gemms the GEMM itself) at the layer's flush
        if (df->gemms) {
            df->gemm.push_back(g.a);
            df->role.push_back(role);
        } else {
            probe_mark(role, false, st, plan);
            U2GNN_TRY(g.run(st, plan));
            probe_mark(role, true, st, plan);
        }
        u2gnn_reduce_job j = rjob(U2GNN_RJOB_SLAB);
        j.src = slabs, j.n_slab = (int32_t)split, j.slab_stride = M * N, j.rows = M, j.cols = N, j.ld_src = N;
        j.rblk_pad = rb0, j.rblk_real = rb1, j.cblk_pad = cb0, j.cblk_real = cb1;
        j.dst = C, j.ld_dst = ldc, j.alpha = alpha, j.accumulate = accumulate ? 1 : 0;
        df->red.push_back(j);
        return U2GNN_OK;
    }
    probe_mark(role, false, st, plan);
    U2GNN_TRY(g.run(st, plan));
    probe_mark(role, true, st, plan);
    if (slabs_out) {   // the consumer sums the slabs itself (u2gnn_layernorm_bwd_delta_slabs)
        *slabs_out = slabs, *nslab_out = split;
        return U2GNN_OK;
    }
    if (plan) return U2GNN_OK;
    hipStream_t rs = st;
    if (red_st && red_st != st) {
        hipEvent_t ev = pooled_event();
        if (!ev) return U2GNN_E_ARG;
        if (hipEventRecord(ev, st) != hipSuccess || hipStreamWaitEvent(red_st, ev, 0) != hipSuccess) return U2GNN_E_ARG;
        rs = red_st;
    }
    return u2gnn_slab_reduce(slabs, (int32_t)split, M * N, M, N, N, rb0, rb1, cb0, cb1, C, ldc, alpha,
                             accumulate ? 1 : 0, rs);
}

// engine._wgrad: dst(real) = unpack(dY^T X)
int wgrad(Arena &W, const Dims &D, const float *dY, int64_t ld_dy, const float *X, int64_t ld_x, int64_t m_pad,
          int64_t n_pad, float *dst, int64_t ld_dst, const int64_t *rblk, const int64_t *cblk, hipStream_t st,
          Defer *df = nullptr) {
    return gemm_split(W, D, dY, X, dst, m_pad, n_pad, D.Np, ld_dy, ld_x, ld_dst, true, 1.f, false, rblk, cblk, true,
                      st, false, -1, 0, nullptr, df);
}

int64_t colstat_ws_floats(int64_t rows, int64_t cols) { return ((rows + 15) / 16 > 0 ? (rows + 15) / 16 : 1) * 3 * cols; }

int bias_grad(Arena &W, const float *dY, int64_t rows, int64_t cols_pad, int64_t ld, int64_t cb0, int64_t cb1,
              float *out, hipStream_t st, Defer *df = nullptr) {
    // taken in both modes: the size plan (u2gnn_layer_sizes runs the one-stream form) covers the side-stream form
    float *ws = W.take<float>(colstat_ws_floats(rows, cols_pad));
    if (df) {
        u2gnn_reduce_job j = rjob(U2GNN_RJOB_COLSUM);
        j.src = dY, j.rows = rows, j.cols = cols_pad, j.ld_src = ld, j.cblk_pad = cb0, j.cblk_real = cb1, j.dst = out;
        df->red.push_back(j);
        return U2GNN_OK;
    }
    if (W.plan()) return U2GNN_OK;
    return u2gnn_colsum(dY, rows, cols_pad, ld, cb0, cb1, out, 0, ws, st);
}

// Fork / join events come from a per-device ring of pre-created events.  Re-recording an event is
// safe once the waits on its previous record are enqueued (a wait binds the record current at the
// call), and a ring of 256 is far longer than the hand-offs of one layer in flight.

// The hand-offs order work of ONE device: no system-scope fence when an event is recorded (the producing
// kernels' own releases make their stores visible to the other queue's kernels).  The record then stops
// holding back the next kernel of the recording stream: dO -> dS gap 13 -> 4.7 us, C4 step 2.963 / 2.958 vs
// 2.987 / 2.978 ms (device-scope release instead: 2.979 / 2.961; profiles/r04/ab_event_fence.txt)
// SAME-DEVICE ONLY: a pooled event may order only two streams of the device it was drawn for (the pools
// are per device, the main and side streams of one layer call share that device).  A cross-device or
// host-visible hand-off must use its own event without hipEventDisableSystemFence.
constexpr unsigned kForkEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;

hipEvent_t pooled_event() {
    constexpr size_t kRing = 256;
    static std::mutex mu;
    static std::map<int, std::pair<std::vector<hipEvent_t>, size_t>> pools;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto &p = pools[dev];
    if (p.first.empty()) {
        p.first.resize(kRing, nullptr);
        for (auto &ev : p.first)
            if (hipEventCreateWithFlags(&ev, kForkEventFlags) != hipSuccess) {
                for (auto &x : p.first)
                    if (x) (void)hipEventDestroy(x);
                p.first.clear();
                return nullptr;
            }
    }
    return p.first[p.second++ % kRing];
}

// side-stream hand-off: the side stream waits for everything issued on main so far
struct Side {
    hipStream_t main, side;
    bool plan;
    int fork() {
        if (plan || side == main) return U2GNN_OK;
        hipEvent_t ev = pooled_event();
        if (!ev) return U2GNN_E_ARG;
        hipError_t e = hipEventRecord(ev, main);
        if (e == hipSuccess) e = hipStreamWaitEvent(side, ev, 0);
        return e == hipSuccess ? U2GNN_OK : (int)e;
    }
    // the main stream waits for everything issued on the side stream so far
    int join() {
        hipEvent_t ev = nullptr;
        U2GNN_TRY(mark(&ev));
        return wait(ev);
    }
    // an event at the side stream's current position (joined later by wait(); nullptr when there
    // is no separate side stream)
    int mark(hipEvent_t *ev) {
        *ev = nullptr;
        if (plan || side == main) return U2GNN_OK;
        *ev = pooled_event();
        if (!*ev) return U2GNN_E_ARG;
        const hipError_t e = hipEventRecord(*ev, side);
        return e == hipSuccess ? U2GNN_OK : (int)e;
    }
    // the main stream waits for a mark() event
    int wait(hipEvent_t ev) {
        if (!ev) return U2GNN_OK;
        const hipError_t e = hipStreamWaitEvent(main, ev, 0);
        return e == hipSuccess ? U2GNN_OK : (int)e;
    }
};

// u2gnn_layernorm_bwd_params now, or as a job of the layer's flush
int ln_params(const float *dY, const float *Z, const float *mean, const float *rstd, const float *dZd, int64_t ld,
              int64_t rows, int64_t d, int64_t dp, float *ws, float *dgamma, float *dbeta, float *dbias, hipStream_t st,
              bool plan, Defer *df) {
    if (df) {
        u2gnn_reduce_job j = rjob(U2GNN_RJOB_LNPARAMS);
        j.src = dY, j.ld_src = ld, j.Z = Z, j.ldz = ld, j.mean = mean, j.rstd = rstd, j.dZdrop = dZd, j.lddrop = ld;
        j.rows = rows, j.d = d, j.cols = dp, j.dst = dgamma, j.dbeta = dbeta, j.dbias = dbias;
        df->red.push_back(j);
        return U2GNN_OK;
    }
    if (plan) return U2GNN_OK;
    return u2gnn_layernorm_bwd_params(dY, ld, Z, ld, mean, rstd, dZd, ld, rows, d, dp, ws, dgamma, dbeta, dbias, st);
}

// Schedule decisions (each measured in rounds 1-2; the A/B switches are gone):
//  * dV = Pd^T dO runs on the side stream beside the dS -> dQ -> dK chain (-1.4 % step time);
//  * LayerNorm forward is fused into the bias-dropout-residual epilogue when one 64-column tile holds
//    whole rows (d <= 64, matrix-core precisions);
//  * delta = rowsum(dO * O) of the attention backward comes from LayerNorm1's backward
//    (u2gnn_layernorm_bwd_delta: sum_c dA * ((Z1 - X)(1-p) - b_o)) in the matrix-core precisions; the
//    fp32 parity path keeps u2gnn_rowdot, whose error does not grow with |X|.
void set_ln(u2gnn_gemm_args &a, const float *gamma, const float *beta, float *y, int64_t ldy, float *mean, float *rstd,
            int64_t d, int64_t rows) {
    a.ln_gamma = gamma, a.ln_beta = beta, a.ln_y = y, a.ln_ldy = ldy;
    a.ln_mean = mean, a.ln_rstd = rstd, a.ln_d = d, a.ln_rows = rows, a.ln_eps = 1e-5f;
}

// the fused attention forward (u2gnn_attn_softmax_pv): node-axis attention in the matrix-core
// precisions with dp <= 384 (engine.fused_attn mirrors the rule)
// split-K depth of FFN2 in the matrix-core precisions (mfma), dp <= 256: with fewer than 128 output
// tiles of 64x64, aim at ~256 blocks of >= 4 K steps; u2gnn_slab_bias_drop_resid_ln then forms the bias,
// dropout, residual and LayerNorm2 (engine.ffn2_split mirrors the rule).  dp = 64 (C5 and the other
// fused-LayerNorm layers) since round 3; dp <= 256 since round 5: C2's IMDBBINARY batches (Np = 128,
// dp = 192) ran FFN2 as 6 blocks of a 32-step K loop, 16 us, plus a LayerNorm launch
int64_t ffn2_split(int64_t dp, bool mfma, int64_t Np, int64_t ffp) {
    const int64_t tiles = (Np / 64) * (dp / 64);
    if (!mfma || dp > 256 || tiles >= 128) return 1;
    int64_t sp = 256 / tiles;
    if (sp > ffp / 128) sp = ffp / 128;
    return sp > 1 ? sp : 1;
}

// tile of S = Q K^T: 256x128 blocks unless they would leave most CUs idle (C5's Np = 2048 gives 128 of
// them), then 128x128 (the same per-element sums: same bits; engine.qk_tile mirrors the rule)
int qk_tile(int64_t Np) { return (Np % 256 == 0 && (Np / 256) * (Np / 128) >= 256) ? 256 : 128; }

// (f16x3 -- the fwdh policy -- runs fused: V as fp16 x2 rows from the in-projection, 3.024 vs 3.052 ms three-pass,
// profiles/r06/h3g_fused_ab.txt; bf16x6 -- the fwd6 policy -- keeps the three-pass form: its fused kernel, ran
// the C4 step at 3.42 / 3.43 ms against 3.40 unfused, and its exp2-based probabilities moved one boundary ReLU unit
// of the test seed's step across 0).  Few rows (C2's IMDBBINARY batches, Np = 128: ONE
// workgroup walks every key) run the three-pass form, whose GEMM tiles spread over more CUs: C2 fwdh 0.424 ms
// three-pass (r6h) vs 0.460 fused (r6i); engine.FUSED_MIN_NP mirrors the bound
constexpr int64_t kFusedMinNp = 1024;
bool fused_attn(const Dims &D) {
#ifdef U2GNN_EXP_H3_UNFUSED   // (A/B: the fwdh policy on the three-pass forward)
    if (D.prec_fwd == U2GNN_PREC_F16X3) return false;
#endif
#ifndef U2GNN_EXP_FUSED_ANY_NP   // (A/B: the fused form at every row count, as up to r6i)
    if (D.Np < kFusedMinNp) return false;
#endif
    return !D.window && !small_attn(D) && D.prec_fwd != U2GNN_PREC_F32 && D.prec_fwd != U2GNN_PREC_BF16X6 &&
           D.dp <= 384;
}

// the row-local tail of a small-width layer (u2gnn_layer_tail_small_*, small_layer.hip): every precision when the
// attention is the small-width one (engine.small_attn mirrors the rule)
u2gnn_small_tail_args tail_args(const Dims &D, const u2gnn_layer_params *w, const u2gnn_layer_seeds *s, const Ctx &c,
                                const float *X, float *X2) {
    u2gnn_small_tail_args t;
    std::memset(&t, 0, sizeof(t));
    t.n_valid = D.N, t.rows_pad = D.Np, t.d = D.d, t.dp = D.dp, t.ff = D.ff, t.ffp = D.ffp;
    t.p = s->p_drop, t.eps = 1e-5f;
    t.seed_drop1 = s->drop1, t.seed_dropff = s->dropff, t.seed_drop2 = s->drop2;
    t.W_o = w->W_o, t.b_o = w->b_o, t.n1_w = w->n1_w, t.n1_b = w->n1_b, t.W1 = w->W1, t.b1 = w->b1;
    t.W2 = w->W2, t.b2 = w->b2, t.n2_w = w->n2_w, t.n2_b = w->n2_b;
    t.O = c.O, t.X = X;
    t.Z1 = c.Z1, t.X1 = c.X1, t.mean1 = c.mean1, t.rstd1 = c.rstd1, t.Hd = c.Hd;
    t.Z2 = c.Z2, t.X2 = X2, t.mean2 = c.mean2, t.rstd2 = c.rstd2;
    return t;
}

int layer_fwd(const Dims &D, const u2gnn_layer_params *w, const u2gnn_layer_seeds *s, const float *X, float *X2,
              Arena &CA, Arena &W, bool need_ctx, hipStream_t st) {
    const int64_t N = D.N, Np = D.Np, d = D.d, dp = D.dp, ffp = D.ffp;
    const int prec = D.prec_fwd;
    const float pd = s->p_drop;
    const bool drop = pd > 0.f;
    const bool plan = W.plan();
    Ctx c = carve_ctx(need_ctx ? CA : W, D, drop);
    const bool fused = fused_attn(D);
    // the in-projection output again in x2 format: the V tiles the fused softmax.P.V kernel reads (bf16x6: it reads
    // the fp32 output itself and splits V in registers, no copy)
    const bool x6 = prec == U2GNN_PREC_BF16X6;
    void *qkv2 = fused && !x6 ? static_cast<void *>(W.take<uint16_t>(Np * 6 * dp)) : nullptr;
    // a3.1 in-projection (+bias, Q scaled by 1/sqrt(d)); the small-width attention does its own
    if (!small_attn(D)) {
        G g(X, w->W_in, c.QKV, Np, 3 * dp, dp, dp, dp, 3 * dp, prec);
        // 256x128 blocks from 3 waves of them on (token-sized rows, neighbour mode), the default tile
        // rule below that: C4's 19 x 9 blocks of 256x128 leave a third of the CUs idle, its 76 x 18 64-tile
        // blocks run the step 0.8 % faster (3/3 reps, profiles/r02/qkv_tile_ab.txt; bit-identical).
        int qkv_tile = (prec != U2GNN_PREC_F32 && Np % 256 == 0 &&
                        (Np / 256) * (3 * dp / 128) >= U2GNN_BIG_TILE_BLOCKS) ? 256 : 0;
#ifdef U2GNN_EXP_QKV256   // (A/B: 256x128 blocks for every in-projection with Np % 256 == 0)
        if (prec != U2GNN_PREC_F32 && Np % 256 == 0) qkv_tile = 256;
#endif
        g.tb().epi(U2GNN_EPI_BIAS).tile(qkv_tile);
        g.a.bias = w->b_in;
        g.a.alpha = (float)(1.0 / std::sqrt((double)d));
        g.a.scale_cols = dp;
        // the x2 copy the fused softmax.P.V kernel reads: its V block only (Q and K are never read in x2)
        if (fused && !x6) g.a.Cx2 = qkv2, g.a.ldcx2 = 6 * dp, g.a.cx2_col0 = (int32_t)(2 * dp);
        U2GNN_TRY(g.run(st, plan));
    }
    const float *Q = c.QKV, *Kt = Q ? Q + dp : nullptr, *V = Q ? Q + 2 * dp : nullptr;   // (no image: small path)
    if (D.window) {
        // paper semantics: attention inside each node's window of W neighbour tokens
        if (!plan)
            U2GNN_TRY(u2gnn_window_attn_fwd(c.QKV, 3 * dp, D.window, (int32_t)dp, c.O, dp, c.Psave, pd, s->attn,
                                            N / D.window, Np, st));
    } else if (small_attn(D)) {
        // d <= 32: the whole layer on the vector ALUs (small_layer.hip): in-projection, softmax -> dropout -> P.V
        // flash-style (the row statistics and a compact Q, K, V saved) and a3.3 + a3.4 -- 2 or 3 launches
        if (!plan) {
            const u2gnn_small_tail_args t = tail_args(D, w, s, c, X, X2);
            probe_mark(U2GNN_ROLE_PV, false, st, plan);
            U2GNN_TRY(u2gnn_layer_small_fwd(&t, w->W_in, w->b_in, s->attn, c.stats, u2gnn_attn_small_ctx_floats(Np, d),
                                            st));
            probe_mark(U2GNN_ROLE_PV, true, st, plan);
        }
    } else if (fused) {
        // a3.2 as S = Q K^T with the softmax row partials from the GEMM epilogue, then one fused
        // softmax -> dropout -> P.V pass that overwrites S with the signed image (attn_fused.hip)
        const int64_t ld_rp = Np / 32, groups = Np / 64;   // 64-column groups of the 256 / 128 tiles
        float *rowpart = W.take<float>(Np * 2 * ld_rp);
        float *pv_ws = W.take<float>(u2gnn_attn_softmax_pv_ws_floats(N, Np, dp));
        {
            G g(Q, Kt, c.Pd, Np, Np, dp, 3 * dp, 3 * dp, Np, prec);
            g.tb().epi(U2GNN_EPI_STORE_ROWSTAT).tile(qk_tile(Np));
            g.a.rowpart = rowpart, g.a.ld_rowpart = ld_rp, g.a.n_valid = N;
            probe_mark(U2GNN_ROLE_QK, false, st, plan);
            U2GNN_TRY(g.run(st, plan));
            probe_mark(U2GNN_ROLE_QK, true, st, plan);
        }
        if (!plan) {
            probe_mark(U2GNN_ROLE_PV, false, st, plan);
            U2GNN_TRY(u2gnn_attn_softmax_pv(c.Pd, Np, rowpart, ld_rp, groups, x6 ? static_cast<const void *>(c.QKV) : qkv2,
                                            x6 ? 3 * dp : 6 * dp, dp, c.Pd, Np, c.O, dp, pv_ws,
                                            u2gnn_attn_softmax_pv_ws_floats(N, Np, dp), N, Np, pd, s->attn, prec, st));
            probe_mark(U2GNN_ROLE_PV, true, st, plan);
        }
    } else {
        // a3.2 scores, softmax + dropout, P.V (fp32 parity path, dp > 384)
        float *S = W.take<float>(Np * Np);
        {
            G g(Q, Kt, S, Np, Np, dp, 3 * dp, 3 * dp, Np, prec);
            g.tb().tile((prec != U2GNN_PREC_F32 && Np % 256 == 0) ? 256 : 0);
            probe_mark(U2GNN_ROLE_QK, false, st, plan);
            U2GNN_TRY(g.run(st, plan));
            probe_mark(U2GNN_ROLE_QK, true, st, plan);
        }
        if (!plan)
            U2GNN_TRY(u2gnn_attn_softmax_fwd(S, Np, drop ? nullptr : c.Pd, c.Pd, Np, N, Np, N, Np, pd, s->attn,
                                             nullptr, 0, st));
        U2GNN_TRY(gemm_split(W, D, c.Pd, V, c.O, Np, dp, Np, Np, 3 * dp, dp, false, 1.f, false, nullptr, nullptr,
                             false, st, drop, prec, U2GNN_ROLE_PV, nullptr, nullptr, nullptr, nullptr,
                             h3_prob_exp(pd)));
    }
    if (small_attn(D)) {
        // a3.3 + a3.4: run by u2gnn_layer_small_fwd above
    } else if (mid_tail(D)) {
        // a3.3 + a3.4 in two launches: out-projection .. FFN2 partials per row block and hidden chunk, then the
        // slab LayerNorm2 (mid_layer.hip)
        const int64_t wsf = u2gnn_layer_tail_mid_ws_floats(Np, dp, ffp);
        float *mws = W.take<float>(wsf > 0 ? wsf : 1);
        if (!plan) {
            const u2gnn_small_tail_args t = tail_args(D, w, s, c, X, X2);
            U2GNN_TRY(u2gnn_layer_tail_mid_fwd(&t, mws, wsf, st));
        }
    } else {
        // a3.3 out-projection + dropout1 + residual, LayerNorm1 (fused into the GEMM epilogue when a
        // 64-column tile holds whole rows: d <= 64, bf16 modes; engine.fused_ln mirrors the rule)
        const bool fuse_ln = dp == 64 && prec != U2GNN_PREC_F32;
        {
            G g(c.O, w->W_o, c.Z1, Np, dp, dp, dp, dp, dp, prec);
            g.tb().epi(fuse_ln ? U2GNN_EPI_BIAS_DROP_RESID_LN : U2GNN_EPI_BIAS_DROP_RESID);
            g.a.bias = w->b_o, g.a.aux0 = X, g.a.ld_aux = dp, g.a.p_drop = pd, g.a.seed = s->drop1;
            if (fuse_ln) set_ln(g.a, w->n1_w, w->n1_b, c.X1, dp, c.mean1, c.rstd1, d, N);
            U2GNN_TRY(g.run(st, plan));
        }
        if (!plan && !fuse_ln)
            U2GNN_TRY(u2gnn_layernorm_fwd(c.Z1, dp, w->n1_w, w->n1_b, c.X1, dp, c.mean1, c.rstd1, N, Np, d, dp, 1e-5f, st));
        // a3.4 FFN + dropout2 + residual, LayerNorm2
        {
            G g(c.X1, w->W1, c.Hd, Np, ffp, dp, dp, dp, ffp, prec);
            g.tb().epi(U2GNN_EPI_BIAS_RELU_DROP);
#ifdef U2GNN_EXP_FFN1_256   // (A/B: FFN1 on 256x128 blocks)
            if (prec != U2GNN_PREC_F32 && Np % 256 == 0 && ffp % 128 == 0) g.tile(256);
#endif
            g.a.bias = w->b1, g.a.p_drop = pd, g.a.seed = s->dropff;
            U2GNN_TRY(g.run(st, plan));
        }
        const int64_t f2_split = ffn2_split(dp, prec != U2GNN_PREC_F32, Np, ffp);
        if (f2_split > 1) {
            // too few output tiles (C5: 32 of them, each a 32-step K loop): split-K slabs, then the
            // bias / dropout / residual / LayerNorm pass over the slabs
            float *slabs = W.take<float>(f2_split * Np * dp);
            G g(c.Hd, w->W2, slabs, Np, dp, ffp, ffp, ffp, dp, prec);
            g.tb().tile(64);
            g.a.split_k = (int32_t)f2_split, g.a.slab_stride = Np * dp;
            U2GNN_TRY(g.run(st, plan));
            if (!plan)
                U2GNN_TRY(u2gnn_slab_bias_drop_resid_ln(slabs, (int32_t)f2_split, Np * dp, dp, w->b2, c.X1, dp, pd,
                                                        s->drop2, c.Z2, dp, w->n2_w, w->n2_b, X2, dp, c.mean2, c.rstd2, d,
                                                        N, Np, 1e-5f, st));
        } else {
            G g(c.Hd, w->W2, c.Z2, Np, dp, ffp, ffp, ffp, dp, prec);
            g.tb().epi(fuse_ln ? U2GNN_EPI_BIAS_DROP_RESID_LN : U2GNN_EPI_BIAS_DROP_RESID);
            g.a.bias = w->b2, g.a.aux0 = c.X1, g.a.ld_aux = dp, g.a.p_drop = pd, g.a.seed = s->drop2;
            if (fuse_ln) set_ln(g.a, w->n2_w, w->n2_b, X2, dp, c.mean2, c.rstd2, d, N);
            U2GNN_TRY(g.run(st, plan));
        }
        if (!plan && !fuse_ln && f2_split <= 1)
            U2GNN_TRY(u2gnn_layernorm_fwd(c.Z2, dp, w->n2_w, w->n2_b, X2, dp, c.mean2, c.rstd2, N, Np, d, dp, 1e-5f, st));
    }
    if ((W.overflow || CA.overflow) && debug_on())
        std::fprintf(stderr, "u2gnn: layer_fwd arena overflow (ws %lld/%lld, ctx %lld/%lld)\n", (long long)W.used,
                     (long long)W.cap, (long long)CA.used, (long long)CA.cap);
    return (W.overflow || CA.overflow) ? U2GNN_E_ARG : U2GNN_OK;
}

int layer_bwd(const Dims &D, const u2gnn_layer_params *w, const u2gnn_layer_seeds *s, const float *X, Arena &CA,
              const float *dX2, float *dX, const u2gnn_layer_grads *g, Arena &W, hipStream_t st, hipStream_t side_st,
              bool need_dx = true) {
    const int64_t N = D.N, Np = D.Np, d = D.d, dp = D.dp, ff = D.ff, ffp = D.ffp;
    const int prec = D.prec;
    const float pd = s->p_drop;
    const bool drop = pd > 0.f;
    const bool plan = W.plan();
    Ctx c = carve_ctx(CA, D, drop);
    Side sd{st, side_st ? side_st : st, plan};
    hipStream_t so = sd.side;
    // The parameter-gradient products and reductions are held back to the end of the layer (df) and go out
    // there as one grouped GEMM launch + one reduction batch: on the side stream, overlapping the next
    // layer's backward (C4: 3.141 / 3.147 / 3.159 vs 3.187 / 3.191 / 3.195 ms per step issued one by one
    // beside this layer, one session, profiles/r03/r3g_side_defer_ab.txt), or on this stream for one-stream
    // layers (C5: -10 launches per layer) and for the last layer of the backward.  The attention products
    // dQ, dK (and dV when it runs on this stream) go out as one grouped launch and their slab reduces as
    // one batch before the in-projection (att; C4 neutral, C5 -2 launches per layer).
    Defer defer_p, defer_a;
    defer_p.gemms = defer_a.gemms = true;
    Defer *df = &defer_p, *att = &defer_a;
    const int64_t blk_d[2] = {dp, d}, blk_ff[2] = {ffp, ff};
    float *ws = W.take<float>(colstat_ws_floats(N, dp));
    const bool tail = small_attn(D);   // the row-local tail kernel (small_layer.hip) forms dX1 ... dO and delta
    // one-stream layers in the matrix-core precisions: LayerNorm1's backward forms delta = rowsum(dO * O)
    const bool ln_delta = !D.window && prec != U2GNN_PREC_F32;
    float *dX1 = W.take<float>(Np * dp), *dF = W.take<float>(Np * dp);
    float *dH = W.take<float>(Np * ffp);
    float *dA = W.take<float>(Np * dp);
    // no input gradient wanted (first layer of the stack): LN1's residual half goes to scratch and
    // the in-projection's dX GEMM below is skipped
    float *dX_scratch = W.take<float>(Np * dp);   // taken in every mode so the plan covers it
    if (!need_dx) dX = dX_scratch;
    float *delta_ln = (ln_delta || tail) ? W.take<float>(Np) : nullptr;
    float *dO = W.take<float>(Np * dp);
    float *small_dqkv = nullptr;   // the small-width layer's dQKV, written by u2gnn_layer_small_bwd
    if (tail) {
        // the tail backward and the attention backward (dQKV; dX += dQKV W_in unless no input gradient is
        // wanted) in 2 or 3 launches (small_layer.hip)
        small_dqkv = W.take<float>(Np * 3 * dp);
        const int64_t wsf = u2gnn_attn_small_ws_floats(N, Np, d);
        float *sa_ws = W.take<float>(wsf);
        if (!plan) {
            u2gnn_small_tail_args t = tail_args(D, w, s, c, X, nullptr);
            t.dX2 = dX2, t.dX1 = dX1, t.dF = dF, t.dH = dH, t.dX = dX, t.dA = dA, t.dO = dO, t.delta = delta_ln;
            probe_mark(U2GNN_ROLE_DS, false, st, plan);
            U2GNN_TRY(u2gnn_layer_small_bwd(&t, w->W_in, s->attn, c.stats, u2gnn_attn_small_ctx_floats(Np, d),
                                            small_dqkv, 3 * dp, need_dx ? 1 : 0, sa_ws, wsf, st));
            probe_mark(U2GNN_ROLE_DS, true, st, plan);
        }
        // the parameter gradients of the tail, held back (df) in the order of the matrix-core branch
        U2GNN_TRY(ln_params(dX2, c.Z2, c.mean2, c.rstd2, dF, dp, N, d, dp, ws, g->n2_w, g->n2_b, g->l2_b, so, plan, df));
        U2GNN_TRY(wgrad(W, D, dF, dp, c.Hd, ffp, dp, ffp, g->l2_w, ff, blk_d, blk_ff, so, df));
        U2GNN_TRY(wgrad(W, D, dH, ffp, c.X1, dp, ffp, dp, g->l1_w, d, blk_ff, blk_d, so, df));
        U2GNN_TRY(bias_grad(W, dH, Np, ffp, ffp, ffp, ff, g->l1_b, so, df));
        U2GNN_TRY(ln_params(dX1, c.Z1, c.mean1, c.rstd1, dA, dp, N, d, dp, ws, g->n1_w, g->n1_b, g->out_b, so, plan, df));
        U2GNN_TRY(wgrad(W, D, dA, dp, c.O, dp, dp, dp, g->out_w, d, blk_d, blk_d, so, df));
    } else {
        // LN2 backward -> dX1 (residual), dF (dropout2 branch); norm2 + linear2.bias grads (held back: df)
        if (!plan)
            U2GNN_TRY(u2gnn_layernorm_bwd(dX2, dp, c.Z2, dp, c.mean2, c.rstd2, w->n2_w, dX1, dp, dF, dp, pd, s->drop2,
                                          N, Np, d, dp, st));
        U2GNN_TRY(ln_params(dX2, c.Z2, c.mean2, c.rstd2, dF, dp, N, d, dp, ws, g->n2_w, g->n2_b, g->l2_b, so, plan, df));
        // FFN
        {
            G gg(dF, w->W2, dH, Np, ffp, dp, dp, ffp, ffp, prec);
            gg.epi(U2GNN_EPI_RELU_DROP_BWD);
            gg.a.aux0 = c.Hd, gg.a.ld_aux = ffp, gg.a.p_drop = pd;
            U2GNN_TRY(gg.run(st, plan));
        }
        U2GNN_TRY(wgrad(W, D, dF, dp, c.Hd, ffp, dp, ffp, g->l2_w, ff, blk_d, blk_ff, so, df));   // held back (df)
        // one-stream layers in the matrix-core precisions: a split-K dX1 product leaves its slabs to LayerNorm1's
        // backward, which completes dX1 before using it (the separate reduce launch goes; same bits)
        float *dx1_slabs = nullptr;
        int64_t dx1_nslab = 0;
        U2GNN_TRY(gemm_split(W, D, dH, w->W1, dX1, Np, dp, ffp, ffp, dp, dp, false, 1.f, true, nullptr, nullptr, false,
                             st, false, -1, 0, nullptr, nullptr, (ln_delta && so == st) ? &dx1_slabs : nullptr,
                             &dx1_nslab));
        U2GNN_TRY(wgrad(W, D, dH, ffp, c.X1, dp, ffp, dp, g->l1_w, d, blk_ff, blk_d, so, df));
        U2GNN_TRY(bias_grad(W, dH, Np, ffp, ffp, ffp, ff, g->l1_b, so, df));
        // LN1 backward -> dX (residual), dA (dropout1 branch); norm1 + out_proj.bias grads (held back: df);
        // node attention: LayerNorm1's backward also forms delta = rowsum(dO * O) for the dS epilogue
        if (!plan && ln_delta && dx1_slabs)
            U2GNN_TRY(u2gnn_layernorm_bwd_delta_slabs(dX1, dp, dx1_slabs, (int32_t)dx1_nslab, Np * dp, c.Z1, dp,
                                                      c.mean1, c.rstd1, w->n1_w, dX, dp, dA, dp, pd, s->drop1, N, Np, d,
                                                      dp, X, dp, w->b_o, delta_ln, st));
        else if (!plan && ln_delta)
            U2GNN_TRY(u2gnn_layernorm_bwd_delta(dX1, dp, c.Z1, dp, c.mean1, c.rstd1, w->n1_w, dX, dp, dA, dp, pd,
                                                s->drop1, N, Np, d, dp, X, dp, w->b_o, delta_ln, st));
        else if (!plan)
            U2GNN_TRY(u2gnn_layernorm_bwd(dX1, dp, c.Z1, dp, c.mean1, c.rstd1, w->n1_w, dX, dp, dA, dp, pd, s->drop1,
                                          N, Np, d, dp, st));
        U2GNN_TRY(ln_params(dX1, c.Z1, c.mean1, c.rstd1, dA, dp, N, d, dp, ws, g->n1_w, g->n1_b, g->out_b, so, plan,
                            df));
        // out-projection
        {
            G gg(dA, w->W_o, dO, Np, dp, dp, dp, dp, dp, prec);
            U2GNN_TRY(gg.run(st, plan));
        }
        U2GNN_TRY(wgrad(W, D, dA, dp, c.O, dp, dp, dp, g->out_w, d, blk_d, blk_d, so, df));   // held back (df)
    }
    const bool have_delta = ln_delta || tail;
    // attention core
    const float *Q = c.QKV, *Kt = Q ? Q + dp : nullptr, *V = Q ? Q + 2 * dp : nullptr;   // (no image: small path)
    const float q_scale = (float)(1.0 / std::sqrt((double)d));
    float *dQKV;
    hipEvent_t dv_done = nullptr;   // side-stream position after the dV product (in_dx waits for it)
    if (D.window) {
        dQKV = W.take<float>(Np * 3 * dp);
        if (!plan)
            U2GNN_TRY(u2gnn_window_attn_bwd(c.QKV, 3 * dp, D.window, (int32_t)dp, dO, dp, c.Psave, pd, s->attn,
                                            q_scale, dQKV, 3 * dp, N / D.window, Np, st));
    } else if (small_attn(D)) {
        // d <= 32: dQ, dK, dV (P recomputed from the row statistics) and dX += dQKV W_in, run with the tail above
        dQKV = small_dqkv;
    } else {
        dQKV = W.take<float>(Np * 3 * dp);
        const bool dv_side = so != st;   // grouped with dQ / dK on this stream instead: 3.136-3.141 vs 3.068-3.098 ms
        // dV needs only Pd and dO: on the side stream it overlaps the dS -> dQ -> dK chain
        U2GNN_TRY(sd.fork());
        U2GNN_TRY(gemm_split(W, D, c.Pd, dO, dQKV + 2 * dp, Np, dp, Np, Np, dp, 3 * dp, true, 1.f, false, nullptr,
                             nullptr, false, dv_side ? so : st, pd > 0.f, -1, U2GNN_ROLE_DV, nullptr,
                             dv_side ? nullptr : att));
        if (dv_side) U2GNN_TRY(sd.mark(&dv_done));
#ifdef U2GNN_EXP_EARLY_FLUSH
        // experiment: the layer's held-back FFN / LayerNorm / out-projection parameter work goes out on the
        // side stream behind dV (beside dS, dQ, dK) instead of at the end of the layer (beside the next
        // layer's FFN backward); only the in-projection's gradients are left for the end
        if (dv_side && need_dx) U2GNN_TRY(flush(df, W, so));   // measured neutral-to-worse (r04 A/B)
#endif
        float *delta = have_delta ? delta_ln : W.take<float>(Np);
        if (!plan && !have_delta) U2GNN_TRY(u2gnn_rowdot(dO, dp, c.O, dp, delta, Np, dp, st));
        float *dS = W.take<float>(Np * Np);
        {
            G gg(dO, V, dS, Np, Np, dp, dp, 3 * dp, Np, D.prec_ab);
            gg.tb().epi(U2GNN_EPI_ATTN_DS_SIGNED);
            gg.a.aux0 = c.Pd, gg.a.rowvec = delta, gg.a.ld_aux = Np, gg.a.p_drop = pd;
            probe_mark(U2GNN_ROLE_DS, false, st, plan);
            U2GNN_TRY(gg.run(st, plan));
            probe_mark(U2GNN_ROLE_DS, true, st, plan);
        }
        U2GNN_TRY(gemm_split(W, D, dS, Kt, dQKV, Np, dp, Np, Np, 3 * dp, 3 * dp, false, q_scale, false, nullptr, nullptr,
                             false, st, false, D.prec_ab, U2GNN_ROLE_DQ, nullptr, att));
        U2GNN_TRY(gemm_split(W, D, dS, Q, dQKV + dp, Np, dp, Np, Np, 3 * dp, 3 * dp, true, 1.f, false, nullptr,
                             nullptr, false, st, false, D.prec_ab, U2GNN_ROLE_DK, nullptr, att));
        U2GNN_TRY(flush(att, W, st));
        U2GNN_TRY(sd.wait(dv_done));   // dV before dX += dQKV W_in
    }
    // in-projection
    if (need_dx && !small_attn(D))
        U2GNN_TRY(gemm_split(W, D, dQKV, w->W_in, dX, Np, dp, 3 * dp, 3 * dp, dp, dp, false, 1.f, true, nullptr,
                             nullptr, false, st));
    U2GNN_TRY(wgrad(W, D, dQKV, 3 * dp, X, dp, 3 * dp, dp, g->in_w, d, blk_d, blk_d, st, df));
    // in_proj_bias: the Q and V thirds are column sums of dQKV; the K third is exactly zero -- a softmax row is
    // invariant to a constant added to its scores, so sum_j dK_j = sum_i Q_i sum_j dS_ij = 0.  The reference's
    // value there is summation noise, which Adam's first step (lr g / (|g| + eps)) turns into moves of up to lr;
    // a column sum over zero rows writes the exact zeros (engine.in_bias_grad mirrors this)
    U2GNN_TRY(bias_grad(W, dQKV, Np, dp, 3 * dp, dp, d, g->in_b, st, df));
    U2GNN_TRY(bias_grad(W, dQKV + dp, 0, dp, 3 * dp, dp, d, g->in_b + d, st, df));
    U2GNN_TRY(bias_grad(W, dQKV + 2 * dp, Np, dp, 3 * dp, dp, d, g->in_b + 2 * d, st, df));
    // the held-back work: on the side stream after everything issued so far, except for the last layer of
    // the backward (need_dx false), where nothing is left to overlap and the hand-off plus the step's final
    // join cost more than the products (C4 round 3: 3.140-3.157 vs 3.171-3.194 ms per step)
    const bool side_flush = so != st && need_dx;
    if (side_flush) U2GNN_TRY(sd.fork());
    U2GNN_TRY(flush(df, W, side_flush ? so : st));
    return (W.overflow || CA.overflow) ? U2GNN_E_ARG : U2GNN_OK;
}

constexpr int32_t FWD_FLAGS = U2GNN_LAYER_FWD_F32 | U2GNN_LAYER_FWD_X6 | U2GNN_LAYER_FWD_H3;
bool dims_ok(const u2gnn_layer_dims *a) {
    return a && a->N >= 1 && a->d >= 1 && a->ff >= 1 && rup(a->d, 64) <= 1024 &&
           (a->precision == U2GNN_PREC_F32 || a->precision == U2GNN_PREC_BF16X3 || a->precision == U2GNN_PREC_BF16) &&
           ((a->flags & FWD_FLAGS) == 0 || a->precision == U2GNN_PREC_BF16X3) &&
           __builtin_popcount((unsigned)(a->flags & FWD_FLAGS)) <= 1 &&   // at most one forward policy
           a->window >= 0 && a->window <= 32 && (a->window == 0 || a->N % a->window == 0);
}

}  // namespace

extern "C" {

int u2gnn_layer_sizes(const u2gnn_layer_dims *dims, float p_drop, int64_t *ctx_bytes, int64_t *fwd_ws_bytes,
                      int64_t *bwd_ws_bytes) {
    if (!dims_ok(dims) || !ctx_bytes || !fwd_ws_bytes || !bwd_ws_bytes) return U2GNN_E_ARG;
    const Dims D = make_dims(dims);
    u2gnn_layer_seeds s;
    std::memset(&s, 0, sizeof(s));
    s.p_drop = p_drop;
    u2gnn_layer_params w;
    std::memset(&w, 0, sizeof(w));
    u2gnn_layer_grads g;
    std::memset(&g, 0, sizeof(g));
    Arena C(nullptr, 0), Wf(nullptr, 0), Wb(nullptr, 0), Cb(nullptr, 0);
    layer_fwd(D, &w, &s, nullptr, nullptr, C, Wf, true, nullptr);
    layer_bwd(D, &w, &s, nullptr, Cb, nullptr, nullptr, &g, Wb, nullptr, nullptr);
    *ctx_bytes = C.used;
    *fwd_ws_bytes = Wf.used;
    *bwd_ws_bytes = Wb.used;
    return U2GNN_OK;
}

int u2gnn_layer_fwd(const u2gnn_layer_dims *dims, const u2gnn_layer_params *w, const u2gnn_layer_seeds *s,
                    const float *X, float *X2, void *ctx, int64_t ctx_bytes, void *ws, int64_t ws_bytes,
                    void *stream) {
    if (!dims_ok(dims) || !w || !s || !X || !X2 || (!ws && ws_bytes > 0)) return U2GNN_E_ARG;
    const Dims D = make_dims(dims);
    // the same call in planning mode first: a workspace or ctx arena smaller than this call takes is
    // refused before anything is launched (never a launch over the end of a caller buffer)
    Arena Pc(nullptr, 0), Pw(nullptr, 0);
    layer_fwd(D, w, s, X, X2, Pc, Pw, ctx != nullptr, reinterpret_cast<hipStream_t>(stream));
    if (Pw.used > (ws ? ws_bytes : 0) || (ctx && Pc.used > ctx_bytes)) return U2GNN_E_ARG;
    static char empty_ws alignas(256)[256];   // a null base would mean "plan only"
    Arena C(ctx, ctx_bytes), W(ws ? ws : empty_ws, ws ? ws_bytes : 0);
    return layer_fwd(D, w, s, X, X2, C, W, ctx != nullptr, reinterpret_cast<hipStream_t>(stream));
}

int u2gnn_layer_bwd(const u2gnn_layer_dims *dims, const u2gnn_layer_params *w, const u2gnn_layer_seeds *s,
                    const float *X, const void *ctx, int64_t ctx_bytes, const float *dX2, float *dX,
                    const u2gnn_layer_grads *g, void *ws, int64_t ws_bytes, void *stream, void *side_stream) {
    if (!dims_ok(dims) || !w || !s || !X || !ctx || !dX2 || !g || (!ws && ws_bytes > 0)) return U2GNN_E_ARG;
    const Dims D = make_dims(dims);
    Arena Pc(nullptr, 0), Pw(nullptr, 0);   // planning pass with this call's schedule (see u2gnn_layer_fwd)
    layer_bwd(D, w, s, X, Pc, dX2, dX, g, Pw, reinterpret_cast<hipStream_t>(stream),
              reinterpret_cast<hipStream_t>(side_stream), dX != nullptr);
    if (Pw.used > (ws ? ws_bytes : 0) || Pc.used > ctx_bytes) return U2GNN_E_ARG;
    static char empty_ws alignas(256)[256];
    Arena C(const_cast<void *>(ctx), ctx_bytes), W(ws ? ws : empty_ws, ws ? ws_bytes : 0);
    return layer_bwd(D, w, s, X, C, dX2, dX, g, W, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<hipStream_t>(side_stream), dX != nullptr);
}

int u2gnn_probe_arm(int32_t role, int32_t capacity) {
    std::lock_guard<std::mutex> lk(g_probe_mu);
    if (g_probe.ev) return U2GNN_E_ARG;   // collect the previous probe first
    if (role < U2GNN_ROLE_QK || role > U2GNN_ROLE_DK || capacity < 1 || capacity > (1 << 16)) return U2GNN_E_ARG;
    hipEvent_t *ev = new hipEvent_t[2 * capacity];
    for (int i = 0; i < 2 * capacity; ++i) {
        // timing events without the system-scope release (the host reads only their timestamps, in
        // u2gnn_probe_collect, after the bench's device synchronize; no data is handed over through them): with
        // it, each mark wrote L2 back and the timed kernel re-fetched its operands -- C4 dS 99.9 -> 89.3 us in
        // rocprof, probe 107.5 -> 93.8 us, step 3.034 -> 3.018 ms (no probe: 3.002; profiles/r05/ab_probe_fence.txt)
        const hipError_t e = hipEventCreateWithFlags(&ev[i], hipEventDisableSystemFence);
        if (e != hipSuccess) {
            for (int j = 0; j < i; ++j) (void)hipEventDestroy(ev[j]);
            delete[] ev;
            return (int)e;
        }
    }
    g_probe.ev = ev, g_probe.cap = capacity, g_probe.n = 0, g_probe.role = role;
    g_probe_role.store(role, std::memory_order_relaxed);
    return U2GNN_OK;
}

int u2gnn_probe_collect(float *total_ms, int32_t *launches) {
    if (!total_ms || !launches) return U2GNN_E_ARG;
    *total_ms = 0.f, *launches = 0;
    std::lock_guard<std::mutex> lk(g_probe_mu);
    if (!g_probe.ev) return U2GNN_OK;
    int rc = U2GNN_OK;
    double tot = 0.0;
    for (int i = 0; i < g_probe.n && rc == U2GNN_OK; ++i) {
        hipError_t e = hipEventSynchronize(g_probe.ev[2 * i + 1]);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, g_probe.ev[2 * i], g_probe.ev[2 * i + 1]);
        if (e != hipSuccess) rc = (int)e;
        tot += ms;
    }
    for (int i = 0; i < 2 * g_probe.cap; ++i) (void)hipEventDestroy(g_probe.ev[i]);
    delete[] g_probe.ev;
    *total_ms = (float)tot, *launches = g_probe.n;
    g_probe = Probe();
    g_probe_role.store(0, std::memory_order_relaxed);
    return rc;
}

}  // extern "C"
