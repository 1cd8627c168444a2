// phg_api.hip -- host side of the C ABI declared in include/phg.h.
//
// Owns the device memory of one scenario batch on one GPU, builds the per-lane ownership layout
// of the PDHG kernel from the shared sparsity pattern, the node / virtual-rank segment tables of
// the PH update kernels, and orders every launch on one HIP stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>
#include <map>

#include "../../include/phg.h"
#include "phg_internal.h"

namespace phg {
int pdhg_num_variants();
void pdhg_variant_shape(int v, int* out6);
hipError_t pdhg_launch(int v, const PdhgArgs& a, hipStream_t stream);
hipError_t prep_launch(const PrepArgs& a, hipStream_t stream);
hipError_t schedule_launch(const int* iters, int S, int unit, int* order, hipStream_t st);
int pdhg_local_num_variants();
void pdhg_local_variant_shape(int v, int* out4);
int pdhg_local_pick_masked(int v, unsigned mb, unsigned mc, unsigned long long bi, unsigned long long bf,
                           unsigned qm);
int pdhg_local_image_items(int v);
hipError_t pdhg_local_image_launch(int v, const PdhgArgs& a, double* img, double* cimg, hipStream_t stream);
void pdhg_local_variant_masks(int v, unsigned* out2);
hipError_t pdhg_local_launch(int v, const PdhgArgs& a, hipStream_t stream);
hipError_t scale_cols_launch(double* cl, double* cu, const double* dc, long cnt, hipStream_t stream);
bool pdhg_local_lone(int v, int S);
int pdhg_local_loop_ops(int v);
size_t pdhg_local_lds_bytes(int v);
int pdhg_block_num_variants();
void pdhg_block_variant_shape(int v, int* out12);
size_t pdhg_block_lds_bytes(int v, int n_pad, int m_pad, int nd, int ecodes);
hipError_t pdhg_block_launch(int v, const PdhgArgs& a, hipStream_t stream);
hipError_t pdhg_stream_launch(const PdhgArgs& a, hipStream_t stream);
hipError_t pdhg_stream_capacity(int* out);
size_t pdhg_stream_lds_bytes(const StreamLayout& L);
hipError_t pdhg_border_launch(const PdhgArgs& a, hipStream_t stream);
size_t pdhg_border_lds_bytes(const BorderLayout& B);
int pdhg_border_max_per_thread();
size_t pdhg_border_granule_words(const BorderLayout& B, const StreamLayout& L);
int pdhg_wave_num_variants();
void pdhg_wave_variant_shape(int v, int* out6);
size_t pdhg_wave_lds_bytes(int v, int wave_doubles);
hipError_t pdhg_wave_launch(int v, const PdhgArgs& a, hipStream_t stream);
int pdhg_mfma_num_variants();
void pdhg_mfma_variant_shape(int v, int* out2);
hipError_t pdhg_mfma_launch(int v, const PdhgArgs& a, hipStream_t stream);
hipError_t piece_gather_launch(const double* vals, int nnz, const int* perm, int E, int S, double* out,
                               hipStream_t st);
hipError_t node_sums_launch(const PhArgs& a, double* nodesum, hipStream_t st);
hipError_t node_sums_head_launch(const PhArgs& a, double* packed, double thr, int first, hipStream_t st);
hipError_t broadcast_row_launch(const double* row, int N, int S, double* out, hipStream_t st);
hipError_t unscale_launch(const double* sv, const double* d, long cnt, double* out, hipStream_t st);
hipError_t w_update_launch(const PhArgs& a, const double* nodesum, double* convpart, hipStream_t st);
hipError_t ph_head_launch(const PhArgs& a, double* packed, double thr, int first, hipStream_t st);
hipError_t ph_step_launch(const PhArgs& a, double* packed, double thr, int first, hipStream_t st);
hipError_t conv_gate_launch(const double* convpart, int P, double* gate, double* gate_host, double seq,
                            hipStream_t st);
hipError_t safe_bound_launch(const PdhgArgs& a, const SafeBoundArgs& b, hipStream_t st);
hipError_t xbar_head_launch(const PhArgs& a, const double* packed, double thr, int first, hipStream_t st);
hipError_t fold_conv_launch(const PhArgs& a, double* convpart, hipStream_t st);
// solves between launch-schedule recomputations (PHG_SCHED_EVERY overrides, for A/B runs)
static int sched_every() {
    static const int v = [] {
        const char* e = getenv("PHG_SCHED_EVERY");
        const int k = e ? atoi(e) : 0;
        return k > 0 ? k : 4;
    }();
    return v;
}
hipError_t eval_obj_launch(int S, int n, int N, const double* x, const double* c, const double* obj_off,
                           const int* nonant_col, const double* xN, const double* W, const double* rho,
                           const double* xbar, const int* xidx, int w_on, int prox_on, double sense,
                           const double* Z, const double* Psm, int smooth_on, double* out, hipStream_t st);
}  // namespace phg

using namespace phg;

static thread_local std::string g_err;

static int fail(const std::string& msg) {
    g_err = msg;
    return -1;
}

#define CK(call)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(std::string(#call) + ": " + hipGetErrorString(e_));                   \
    } while (0)


struct phg_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool loaded = false;
    // the solves store only the scaled state (xs, ys); the unscaled x / y (x_out, y_out) are
    // materialised from it when something reads them (materialize_outputs)
    bool out_stale = false;
    int S = 0, n = 0, m = 0, nnz = 0, N = 0, L = 0, N_tot = 0, n_nodes = 0, P = 1, n_pad = 0;
    double sense = 1.0;
    int variant = -1;          // gather kernel variant (pdhg.hip), or
    int local_variant = -1;    // lane-local kernel variant (pdhg_local.hip); preferred when >= 0
    // the variant for solves that do not fix the nonants (phg_opts.fix_nonants == 0): its finite
    // bound sides may include rows of nonants only, which fixing frees (local_fin_mask)
    int local_variant_free = -1;
    int local_shape_v = -1;    // its shape's generic entry (pdhg_local_pick_masked re-picks from it)
    std::vector<int> lp_col_of, lp_row_of, lp_cpl_row;   // host copy of the lane plan (bound masks)
    // host copy of the presolved batch: the safe-bound pass's implied bounds are computed from it at
    // the first safe-bound solve (not at every load) and again after phg_set_col_bounds
    struct {
        std::vector<int> rowptr, colidx, nonant_col;
        std::vector<double> vals, rl, ru, cl, cu;
    } hb;
    std::vector<int> fold_col;            // presolve-folded rows as column bounds (Presolved)
    std::vector<double> fold_lo, fold_hi;
    bool sb_stale = true;
    int block_variant = -1;    // workgroup-per-scenario kernel variant (pdhg_block.hip)
    int wave_variant = -1;     // one-wave-per-scenario shared-matrix kernel variant (pdhg_wave.hip)
    int wshape[6] = {0};
    WaveLayout wv{};
    std::vector<int> wave_rperm, wave_cperm;   // piece / column-entry layout -> CSR position
    int mfma_variant = -1;     // shared-matrix MFMA kernel variant (pdhg_mfma.hip)
    bool stream_layout = false;   // multi-workgroup streaming kernel (pdhg_stream.hip)
    bool border_layout = false;   //   ... its bordered block-diagonal form (pdhg_border.hip)
    BorderLayout bd{};
    StreamLayout st{};
    std::vector<int> stream_cperm;   // CSC entry -> CSR position (values gathered after prep)
    int mshape[2] = {0, 0};
    MfmaLayout mf{};
    int bshape[12] = {0};
    std::vector<int> block_rperm, block_cperm;   // piece layout -> CSR position (host copies)
    bool vals_shared = false;
    // delta value form (phg_batch.vals_form): vary[p] = CSR position p differs between scenarios;
    // delta_scale = the workgroup kernel holds the unscaled constant entries once and applies each
    // scenario's scaling on the fly (BlockLayout::vscale), streaming only the entry rows that vary
    std::vector<char> vary;
    int n_vary = 0;
    bool delta_scale = false;
    int layout_policy = PHG_LAYOUT_AUTO;
    int vshape[6] = {0};
    int lshape[4] = {0};
    unsigned local_masks[2] = {0, 0};   // occupied block / coupling slots of the lane-local layout
    std::vector<void*> allocs;
    // device arrays
    double *vals = nullptr, *c = nullptr, *cl = nullptr, *cu = nullptr, *rl = nullptr, *ru = nullptr;
    double *dc = nullptr, *dr = nullptr, *eta = nullptr, *bnorm = nullptr, *obj_off = nullptr;
    double *W = nullptr, *rho = nullptr, *xbar = nullptr, *xsqbar = nullptr, *fixed = nullptr;
    double *Z = nullptr, *Psm = nullptr, *beta = nullptr;   // smoothed PH
    int smooth_on = 0;
    int* xidx = nullptr;
    double *xs = nullptr, *ys = nullptr, *omega = nullptr, *x_out = nullptr, *y_out = nullptr;
    double *xN = nullptr, *obj = nullptr, *bound = nullptr, *kkt = nullptr, *eval = nullptr;
    int *iters = nullptr, *status = nullptr;
    // Solve state is double-buffered: a solve reads the "front" copy (warm start) and writes the
    // "back" copy, then the two are swapped.  So the state before the last solve survives it, which
    // is what lets the PH iteration be speculative by one solve (phg_ph_head): a solve found to be
    // past convergence is undone by swapping back (phg_solve_undo), and a solve gated off on the
    // device writes nothing, so its own swap restores the state before the previous solve.
    struct SolveState {
        double *xs, *ys, *omega, *xN, *obj, *bound, *kkt;
        int *iters, *status;
    } back{};
    int swaps = 0;             // solves since load (parity of the front copy; phg_solve_undo)
    int* order = nullptr;      // launch schedule (schedule.hip)
    unsigned* queue = nullptr; // work queue of the persistent lane-local kernel
    bool persist = false;      // PHG_LOCAL_PERSIST=1 selects the persistent work-queue grid (measured slower)
    // PHG_AVG_EVERY: the lane-local kernel evaluates the average iterate at every avg_every-th
    // check only (restarts / termination on the current iterate otherwise).  Farmer 10k A/B on the
    // box: 1 -> 26.7 M solves/s (272.7 PDHG iterations per solve), 3 -> 27.4 M, 6 -> 27.9 M
    // (283.6), never -> 28.1 M (283.2): the average's products are ~half of a check's work, and on
    // these warm-started prox-QPs the current iterate restarts about as well.  Round 5 (farmer 10k,
    // 4 A/B pairs): 12 -> 0.2834-0.2896 vs 0.2863-0.2939 ms per PH iteration at 6, time to conv
    // 0.801-0.805 vs 0.821-0.829 s, the same 5 185 PH iterations and EF gaps (24: within noise of
    // 6).  12 (every 384th PDHG iteration) keeps the average in reach of long (cold, LP) solves.
    int avg_every = 12;
    // PHG_FUSE=1: phg_ph_step runs node sums + W update as ONE launch (ph_step_kernel) where the batch
    // allows.  Off by default: on farmer 10k the fused launch took 23.7 us against 18.4 us for the two
    // launches back to back (its last-K hand-offs cost more than the launch and the x re-read save),
    // 0.364 vs 0.361 ms per PH iteration; same bits either way (test_pipelined_iteration_matches_sequential)
    bool no_fuse = true;
    bool have_order = false;
    // a launch schedule due (the last solve's iteration counts, sched_src, in units of sched_unit):
    // carried by the next HEADX node-sum launch (phg_ph_step) or, if a solve comes first, launched
    // on its own just before it (sched_flush) -- either way it runs between the two solves, as a
    // launch right behind the solve would
    bool sched_pending = false;
    const int* sched_src = nullptr;
    int sched_unit = 1;
    double* pinned = nullptr;  // page-locked readback buffer (convergence partials)
    // page-locked staging of phg_set's uploads (a ring: each slot reused once its copy has run, so
    // phg_set returns without a stream synchronisation) and of phg_solve_results' one readback
    struct Stage { void* p = nullptr; size_t cap = 0; hipEvent_t ev = nullptr; };
    Stage up[4];
    int up_next = 0;
    Stage down;
    int summary[2] = {0, 0};   // scenarios not optimal / NaN, as of the last phg_conv_finish
    int* nonant_col_d = nullptr;
    unsigned char* row_fixed = nullptr;   // [m] every column of the (kept) row is a nonant
    Layout lay{};
    LocalLayout loc{};
    BlockLayout blk{};
    PhArgs ph{};
    // the one cross-GPU exchange buffer: [2*N_tot node sums | 2P+2 convergence / status partials |
    // 1 flag (> 0: the partials hold a W update's values)] -- one all-reduce per PH iteration
    double *packed = nullptr, *nodesum = nullptr, *convpart = nullptr;
    std::vector<int> nonant_col_h;
    // timing of the last launches (HIP events on the handle's stream)
    // per-launch timing since the last phg_timing_reset: event pairs of every solve (0) and every
    // PH update (1), read only when phg_timing is called -- no per-launch host synchronisation
    // (2: node sums alone, 3: the W update / head alone; a PH update = node sums + W update, timed
    // from the node sums' begin to the W update's end, which = 1)
    std::vector<hipEvent_t> tev[4];
    int tcount[4] = {0, 0, 0, 0};
    bool t_open = false;       // a PH update's begin event is recorded, its end not yet
    int timing_mask = 0;       // bit 0: time solves, bit 1: time PH updates (and their two kernels)
    long long* iters_acc = nullptr;
    // singleton-row presolve (presolve_singletons): rows of the caller's batch -> kept rows
    int presolve = 1;
    int m_orig = 0;
    // device-side convergence metric (phg_conv_start / phg_conv_wait, predicated solves)
    double* gate = nullptr;          // device {conv, not optimal, NaN}
    double* gate_host = nullptr;     // fine-grained pinned host ring [2][4]: slot seq mod 2 = {values, seq}
    long long gate_seq = 0;          // sequence number of the last enqueued gate computation
    long long wait_seq = 0;          // the one phg_conv_wait waits for (a tail's gate: not yet)
    long long last_wait_seq = 0;     // the last one waited for, and its conv value
    double last_conv = 0.0;
    bool gate_fused = false;         // the last phg_apply_xbar already computed the gate
    // PH update fused into the end of the next solve (ph_tail.h; phg_set_tail): the request for the
    // next phg_solve, and the last solve's tail whose results phg_ph_step / phg_node_sums take over
    // when that solve ran (it was gated on the gate published as gated_seq: the host has waited for
    // that value and it was not below gate_below)
    int tail_req = 0;
    double tail_req_thr = 0.0;
    double* tail_req_out = nullptr;
    struct {
        int mode = 0;
        double thr = 0.0, gate_below = 0.0;
        long long gated_seq = 0, seq = 0;
        double* out = nullptr;
    } tp;
    // the tail's unit counters, scenario -> unit maps and final slot plan (TailArgs; build_ph_tables)
    unsigned* tail_segcnt = nullptr;
    unsigned* tail_csegcnt = nullptr;
    unsigned* tail_done = nullptr;
    int* tail_scen_seg = nullptr;
    int* tail_scen_cseg = nullptr;
    int* tail_fin = nullptr;
    int tail_nfin = 0;
    double* xbar_next = nullptr;     // [2 N_tot] staging x-bar of the one-GPU tail
    // the launch schedule is recomputed after every sched_every()-th solve (iteration counts move
    // slowly under warm starts; the sort is a latency-bound single-workgroup launch)
    int solves = 0;
    double* rho_k = nullptr;   // [N] copy of rho when it is the same in every scenario (PhArgs::rho_k)
    std::vector<int> row_map;  // original row -> kept row, or -1 (folded into a column bound)
    // phg_opts.safe_bound (bound.hip): pattern, implied column bounds, repair candidates; the
    // scratch (SafeBoundArgs::Y, R) is allocated at the first safe-bound solve
    SafeBoundArgs sb{};
    // relative-gap test on the whole objective (PdhgArgs::gap_const); PHG_GAP_RAW=1 turns it off
    int gap_const = 1;
    // PdhgArgs::sum_stride: 2, the only form the lane-local kernel compiles (end of round 4; the
    // every-iterate and windowed loops and PHG_SUM_STRIDE are gone).  Since round 4 the average iterate's
    // running sums take every second iterate -- farmer 10k: 0.268 vs 0.285 ms per PDHG launch (7 of
    // ~62 instructions per PDHG iteration saved in every other iteration), the same 286 PDHG
    // iterations per solve, time to conv 0.845 vs 0.852 s; round 3 measured it within noise
    int sum_stride = 2;
    // folded PH update (phg_ph_head -> the next phg_solve's prologue does Update_W), lane-local
    // layout without smoothing / variable probability.  ON by default since round 4 (PHG_FOLD=0 /
    // phg_set_fold turn it off): the branch-free prologue loads W with the scenario's other data, so
    // the fold no longer lengthens the PDHG launch (farmer 10k: 0.2851 ms either way) and it drops the
    // W-update launch and its second read of x (0.3108 vs 0.3138 ms per PH iteration, time to conv
    // 0.850 vs 0.864 s); round 3 (dependent prologue chain) measured it 9 us slower on farmer
    int fold = -1;             // -1: on (phg_load_batch), unless PHG_FOLD / phg_set_fold said otherwise
    bool fold_w_pending = false;      // xbar of update k is in place, its W update not yet applied
    bool xn_external = false;         // PHG_F_XN was set by the caller: xN != xs dc until the next solve
    bool fold_conv_pending = false;   // the last solve did a folded update: its conv partials are
                                      // per scenario (conv_s / fold_st), not yet in any partials buffer
    double fold_thr = 0.0;            // convthresh of the head that left fold_w_pending (flush_fold's gate)
    bool flushed_partials = false;    // flush_fold wrote its conv partials into the handle's own buffer;
                                      // the next phg_node_sums / phg_fold_partials into a caller's
                                      // exchange buffer copies them there
    double* conv_s = nullptr;
    int* fold_st = nullptr;
};

template <class T>
static int dalloc(phg_handle* h, T** p, size_t count) {
    void* q = nullptr;
    if (count == 0) count = 1;
    CK(hipMalloc(&q, count * sizeof(T)));
    CK(hipMemsetAsync(q, 0, count * sizeof(T), h->stream));
    h->allocs.push_back(q);
    *p = (T*)q;
    return 0;
}

template <class T>
static int dput(phg_handle* h, T** p, const T* src, size_t count) {
    if (dalloc(h, p, count)) return -1;
    if (src) CK(hipMemcpyAsync(*p, src, count * sizeof(T), hipMemcpyHostToDevice, h->stream));
    return 0;
}

static int timing_event(phg_handle* h, int which, int half) {
    if (!(h->timing_mask & (1 << (which >= 2 ? 1 : which)))) return 0;
    std::vector<hipEvent_t>& v = h->tev[which];
    const size_t idx = 2 * (size_t)h->tcount[which] + half;
    while (v.size() <= idx) {
        hipEvent_t e;
        // timing only: no system-scope fence (the launch's own end-of-kernel release already
        // orders the data for the next launch; nothing here is read by the host through the event)
        CK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        v.push_back(e);
    }
    CK(hipEventRecord(v[idx], h->stream));
    if (half == 1) h->tcount[which]++;
    return 0;
}

static int materialize_outputs(phg_handle* h) {
    if (!h->out_stale) return 0;
    CK(hipSetDevice(h->device));
    CK(unscale_launch(h->xs, h->dc, (long)h->S * h->n, h->x_out, h->stream));
    CK(unscale_launch(h->ys, h->dr, (long)h->S * h->m, h->y_out, h->stream));
    h->out_stale = false;
    return 0;
}

// the folded update applies to this handle's solves (PdhgArgs::fold_w): lane-local layout, W kept
// for every nonant (no variable-probability mask), no smoothing centre to update
static bool fold_active(const phg_handle* h) {
    return h->fold > 0 && h->local_variant >= 0 && !h->smooth_on && !h->ph.pcv;
}

// a folded W update whose solve has not run (xbar of update k in place, phg_ph_head done): apply it
// now with the standalone kernel (W, and its conv partials into the handle's own buffer) -- for
// anything that reads or rewrites W, or a second head before a solve
// (gated like the head that left it pending -- nothing moves when that head found conv
// below its convthresh -- and its partials, written to the handle's own buffer, are carried into the
// caller's exchange buffer by the next phg_node_sums / phg_fold_partials instead of being lost, which
// would leave that buffer's already all-reduced partials to be summed a second time)
// the last solve's fused tail ran (ph_tail.h): that solve was predicated on the gate the host has
// since waited for, and the value was not below its threshold (a gated-off launch runs nothing)
static bool tail_ran(const phg_handle* h) {
    return h->tp.mode != 0 && h->last_wait_seq == h->tp.gated_seq && h->last_conv >= h->tp.gate_below;
}

static int flush_fold(phg_handle* h) {
    if (!h->fold_w_pending) return 0;
    PhArgs a = h->ph;
    a.skip_gate = h->gate;
    a.skip_below = h->fold_thr;
    CK(w_update_launch(a, h->xbar, h->convpart, h->stream));
    h->fold_w_pending = false;
    h->fold_conv_pending = false;
    h->flushed_partials = true;
    return 0;
}

// flushed partials into a caller's partials region (dst: the exchange buffer's, or null = the handle's
// own, where they already are)
static int carry_flushed_partials(phg_handle* h, double* dst) {
    if (!h->flushed_partials) return 0;
    h->flushed_partials = false;
    if (!dst || dst == h->convpart) return 0;
    // the 2P+2 partials and the flag a W update sets (convpart[2P+2])
    CK(hipMemcpyAsync(dst, h->convpart, (2 * (size_t)h->P + 3) * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    return 0;
}

// front <-> back copy of the solve state (see phg_handle::SolveState)
static void swap_state(phg_handle* h) {
    std::swap(h->xs, h->back.xs);
    std::swap(h->ys, h->back.ys);
    std::swap(h->omega, h->back.omega);
    std::swap(h->xN, h->back.xN);
    std::swap(h->obj, h->back.obj);
    std::swap(h->bound, h->back.bound);
    std::swap(h->kkt, h->back.kkt);
    std::swap(h->iters, h->back.iters);
    std::swap(h->status, h->back.status);
    h->ph.xN = h->xN;          // the PH update kernels read the front copy
    h->ph.status = h->status;
    h->out_stale = true;
}

// the due launch schedule on a launch of its own (phg_handle::sched_pending)
// largest shard whose launch schedule rides in the node-sum launch (phg_ph_step): measured up to
// farmer 10 000 (the head with the sort 16.0 us on average against 13.6 + 11.1 us every 4th
// iteration for the two launches; time to conv 0.775 / 0.776 vs 0.781 / 0.780 s); beyond 16 384 the
// 1 024-thread launch (unmeasured there)
constexpr int kSchedFuseMaxS = 16384;

static int sched_flush(phg_handle* h) {
    if (!h->sched_pending) return 0;
    h->sched_pending = false;
    CK(schedule_launch(h->sched_src, h->S, h->sched_unit, h->order, h->stream));
    h->have_order = true;
    return 0;
}

extern "C" {

const char* phg_last_error(void) { return g_err.c_str(); }

int phg_create(int device, phg_handle** out) {
    if (!out) return fail("phg_create: out is NULL");
    int ndev = 0;
    CK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail("phg_create: bad device index");
    CK(hipSetDevice(device));
    phg_handle* h = new phg_handle();
    h->device = device;
    // (PHG_LOCAL_PERSIST, the persistent work-queue grid, is no longer honoured: measured slower in
    // round 1 and found to hang in round 4 -- the kernel's gate return skips its queue re-arm)
    if (const char* ev = std::getenv("PHG_AVG_EVERY")) h->avg_every = std::max(1, std::atoi(ev));
    if (const char* ev = std::getenv("PHG_FUSE")) h->no_fuse = std::atoi(ev) == 0;
    if (const char* ev = std::getenv("PHG_GAP_RAW")) h->gap_const = std::atoi(ev) == 0;
    if (const char* ev = std::getenv("PHG_FOLD")) h->fold = std::atoi(ev) != 0 ? 1 : 0;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return fail("phg_create: hipStreamCreate failed");
    }
    h->own_stream = true;
    *out = h;
    return 0;
}

void phg_destroy(phg_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    for (void* p : h->allocs) (void)hipFree(p);
    if (h->pinned) (void)hipHostFree(h->pinned);
    if (h->gate_host) (void)hipHostFree(h->gate_host);
    for (auto& st : h->up) {
        if (st.p) (void)hipHostFree(st.p);
        if (st.ev) (void)hipEventDestroy(st.ev);
    }
    if (h->down.p) (void)hipHostFree(h->down.p);
    for (auto& v : h->tev)
        for (auto& e : v) (void)hipEventDestroy(e);
    if (h->own_stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int phg_set_stream(phg_handle* h, void* s) {
    if (!h) return fail("null handle");
    CK(hipSetDevice(h->device));
    if (h->own_stream) {
        CK(hipStreamSynchronize(h->stream));
        CK(hipStreamDestroy(h->stream));
        h->own_stream = false;
    }
    h->stream = (hipStream_t)s;
    return 0;
}

static double* field_ptr(phg_handle* h, int f, size_t* count);

// ------------------------------------------------------------------------------ cylinders
// Device-to-device hand-offs between handles on the same GPU (hub -> spoke), ordered across
// their streams by events in BOTH directions: the copy on dst's stream waits for src's work so far,
// and src's later work waits for the copy (src's buffers are rewritten in place by its next W
// update / solve; without the second wait a spoke could read a W torn between two PH iterations).
static int cross_stream_wait(phg_handle* dst, phg_handle* src) {
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, src->stream));
    CK(hipStreamWaitEvent(dst->stream, e, 0));
    CK(hipEventDestroy(e));
    return 0;
}

int phg_copy_from(phg_handle* dst, phg_handle* src, int32_t field) {
    if (!dst || !src || !dst->loaded || !src->loaded) return fail("phg_copy_from: handles not loaded");
    if (dst->device != src->device) return fail("phg_copy_from: handles on different devices");
    if (field == PHG_F_WARM) {
        // src's last solution as dst's warm start: the scaled front state (same batch -> the same
        // deterministic scaling on both handles) and its primal weights
        if (dst->S != src->S || dst->n != src->n || dst->m != src->m)
            return fail("phg_copy_from: PHG_F_WARM needs the same batch on both handles");
        CK(hipSetDevice(dst->device));
        if (cross_stream_wait(dst, src)) return -1;
        CK(hipMemcpyAsync(dst->xs, src->xs, (size_t)dst->S * dst->n * sizeof(double), hipMemcpyDeviceToDevice, dst->stream));
        CK(hipMemcpyAsync(dst->ys, src->ys, (size_t)dst->S * dst->m * sizeof(double), hipMemcpyDeviceToDevice, dst->stream));
        CK(hipMemcpyAsync(dst->omega, src->omega, (size_t)dst->S * sizeof(double), hipMemcpyDeviceToDevice, dst->stream));
        dst->out_stale = true;
        return cross_stream_wait(src, dst);
    }
    if (flush_fold(src) || flush_fold(dst)) return -1;
    size_t nd = 0, ns = 0;
    double* pd = field_ptr(dst, field, &nd);
    double* ps = field_ptr(src, field, &ns);
    if (!pd || !ps) return fail("phg_copy_from: unknown field");
    if (nd != ns) return fail("phg_copy_from: field sizes differ (different batches)");
    if (field == PHG_F_X || field == PHG_F_Y) {
        if (materialize_outputs(src) || materialize_outputs(dst)) return -1;
    }
    CK(hipSetDevice(dst->device));
    if (cross_stream_wait(dst, src)) return -1;
    CK(hipMemcpyAsync(pd, ps, nd * sizeof(double), hipMemcpyDeviceToDevice, dst->stream));
    if (field == PHG_F_RHO) {   // dst's rho is now src's: so is its shared [N] copy (or its absence)
        if (src->ph.rho_k && !dst->rho_k) {
            double* q;
            if (dalloc(dst, &q, (size_t)std::max(1, dst->N))) return -1;
            dst->rho_k = q;
        }
        if (src->ph.rho_k)
            CK(hipMemcpyAsync(dst->rho_k, src->ph.rho_k, (size_t)dst->N * sizeof(double), hipMemcpyDeviceToDevice,
                              dst->stream));
        dst->ph.rho_k = src->ph.rho_k ? dst->rho_k : nullptr;
    }
    // and the other direction: src's next work (e.g. the hub's W update, which rewrites W in place)
    // must not start before the copy has read src's buffer
    return cross_stream_wait(src, dst);
}

int phg_fix_from(phg_handle* dst, phg_handle* src, int32_t scen) {
    if (!dst || !src || !dst->loaded || !src->loaded) return fail("phg_fix_from: handles not loaded");
    if (dst->L != 1 || src->N != dst->N) return fail("phg_fix_from: two-stage batches with equal nonant counts only");
    if (scen < 0 || scen >= src->S) return fail("phg_fix_from: scenario index out of range");
    CK(hipSetDevice(dst->device));
    if (cross_stream_wait(dst, src)) return -1;
    // fixed[s, :] = src.xN[scen, :] for every s (same device: read straight from src's buffer)
    CK(broadcast_row_launch(src->xN + (size_t)scen * src->N, dst->N, dst->S, dst->fixed, dst->stream));
    // src's next solve rewrites xN: it waits for the broadcast to have read the candidate row
    return cross_stream_wait(src, dst);
}

int phg_query(phg_handle* h, int32_t* idle) {
    if (!h) return fail("null handle");
    const hipError_t e = hipStreamQuery(h->stream);
    if (e == hipSuccess) { *idle = 1; return 0; }
    if (e == hipErrorNotReady) { *idle = 0; return 0; }
    return fail(std::string("phg_query: ") + hipGetErrorString(e));
}

int phg_set_smoothing(phg_handle* h, int32_t on) {
    if (!h || !h->loaded) return fail("phg_set_smoothing: no batch loaded");
    h->smooth_on = on ? 1 : 0;
    h->ph.smooth_on = h->smooth_on;
    return 0;
}

int phg_set_layout(phg_handle* h, int32_t policy) {
    if (!h) return fail("null handle");
    if (h->loaded) return fail("phg_set_layout: must be called before phg_load_batch");
    if (policy < PHG_LAYOUT_AUTO || policy > PHG_LAYOUT_WAVE) return fail("phg_set_layout: bad policy");
    h->layout_policy = policy;
    return 0;
}

int phg_sync(phg_handle* h) {
    if (!h) return fail("null handle");
    CK(hipStreamSynchronize(h->stream));
    return 0;
}

// ------------------------------------------------------------------------------ batch loading
static int build_layout(phg_handle* h, const phg_batch* b, const std::vector<int>& colptr,
                        const std::vector<int>& csc_row, const std::vector<int>& csc_p) {
    const int n = b->n, m = b->m;
    int kcs_need = 0;
    for (int j = 0; j < n; ++j) kcs_need = std::max(kcs_need, colptr[j + 1] - colptr[j]);
    const int cpl_need = (n + 63) / 64, rpl_need = (m + 63) / 64;
    int chosen = -1;
    int sh[6];
    for (int v = 0; v < pdhg_num_variants(); ++v) {
        pdhg_variant_shape(v, sh);
        const int CPL = sh[0], KCS = sh[1], RPL = sh[2], KRS = sh[3], D = sh[4], KD = sh[5];
        if (CPL < cpl_need || RPL < rpl_need || KCS < kcs_need) continue;
        int nd = 0, maxd = 0;
        for (int i = 0; i < m; ++i) {
            const int len = b->rowptr[i + 1] - b->rowptr[i];
            if (len > KRS) { ++nd; maxd = std::max(maxd, len); }
        }
        if (nd > D || (maxd + 63) / 64 > KD) continue;
        chosen = v;
        break;
    }
    if (chosen < 0) {
        char msg[256];
        snprintf(msg, sizeof msg,
                 "phg_load_batch: no PDHG kernel variant fits n=%d m=%d max col nnz=%d "
                 "(wave-per-scenario variants cover n,m <= 256)", n, m, kcs_need);
        g_err = msg;
        return 1;
    }
    pdhg_variant_shape(chosen, sh);
    const int CPL = sh[0], KCS = sh[1], RPL = sh[2], KRS = sh[3], D = sh[4], KD = sh[5];
    h->variant = chosen;
    std::memcpy(h->vshape, sh, sizeof sh);
    std::vector<int> col_of(64 * CPL, -1), cent_p(64 * CPL * KCS, -1), cent_row(64 * CPL * KCS, 0);
    for (int j = 0; j < n; ++j) {
        const int ln = j % 64, sl = j / 64;
        col_of[ln * CPL + sl] = j;
        int t = 0;
        for (int e = colptr[j]; e < colptr[j + 1]; ++e, ++t) {
            cent_p[(ln * CPL + sl) * KCS + t] = csc_p[e];
            cent_row[(ln * CPL + sl) * KCS + t] = csc_row[e];
        }
    }
    std::vector<int> row_of(64 * RPL, -1), row_dense(64 * RPL, -1), rent_p(64 * RPL * KRS, -1),
        rent_col(64 * RPL * KRS, 0);
    std::vector<int> dent_p(std::max(1, D * 64 * KD), -1), dent_col(std::max(1, D * 64 * KD), 0);
    int nd = 0;
    for (int i = 0; i < m; ++i) {
        const int ln = i % 64, sl = i / 64;
        row_of[ln * RPL + sl] = i;
        const int len = b->rowptr[i + 1] - b->rowptr[i];
        if (len > KRS) {
            row_dense[ln * RPL + sl] = nd;
            for (int e = 0; e < len; ++e) {
                const int p = b->rowptr[i] + e;
                const int dl = e % 64, t = e / 64;
                dent_p[(nd * 64 + dl) * KD + t] = p;
                dent_col[(nd * 64 + dl) * KD + t] = b->colidx[p];
            }
            ++nd;
        } else {
            for (int e = 0; e < len; ++e) {
                const int p = b->rowptr[i] + e;
                rent_p[(ln * RPL + sl) * KRS + e] = p;
                rent_col[(ln * RPL + sl) * KRS + e] = b->colidx[p];
            }
        }
    }
    int* p;
    if (dput(h, &p, col_of.data(), col_of.size())) return -1; h->lay.col_of = p;
    if (dput(h, &p, cent_p.data(), cent_p.size())) return -1; h->lay.cent_p = p;
    if (dput(h, &p, cent_row.data(), cent_row.size())) return -1; h->lay.cent_row = p;
    if (dput(h, &p, row_of.data(), row_of.size())) return -1; h->lay.row_of = p;
    if (dput(h, &p, row_dense.data(), row_dense.size())) return -1; h->lay.row_dense = p;
    if (dput(h, &p, rent_p.data(), rent_p.size())) return -1; h->lay.rent_p = p;
    if (dput(h, &p, rent_col.data(), rent_col.size())) return -1; h->lay.rent_col = p;
    if (dput(h, &p, dent_p.data(), dent_p.size())) return -1; h->lay.dent_p = p;
    if (dput(h, &p, dent_col.data(), dent_col.size())) return -1; h->lay.dent_col = p;
    return 0;
}

// Lane-local layout (pdhg_local.hip): pick coupling rows greedily (longest row of an oversized
// block) until every connected block of the remaining row/column graph fits one lane (<= CPL
// columns, <= RPL rows), then first-fit-decreasing pack the blocks into LPS lanes.
// Returns 0 (built), 1 (this shape does not fit), -1 (error).
struct LocalPlan {
    std::vector<int> col_of, row_of, blk_p, cpl_row, cpl_p;
};

static int plan_local(const phg_batch* b, int LPS, int CPL, int RPL, int D, LocalPlan& P) {
    const int n = b->n, m = b->m;
    if (n > LPS * CPL || m > LPS * RPL + D) return 1;
    std::vector<char> coupling(m, 0);
    std::vector<int> cpl;
    std::vector<int> par(n);
    std::vector<int> comp_of_col(n), comp_of_row(m);
    int ncomp = 0;
    std::vector<int> ccols, crows;
    // connected blocks of the graph without the coupling rows (and without row `skip`)
    auto blocks = [&](int skip) {
        for (int j = 0; j < n; ++j) par[j] = j;
        auto find = [&](int j) { while (par[j] != j) { par[j] = par[par[j]]; j = par[j]; } return j; };
        for (int i = 0; i < m; ++i) {
            if (coupling[i] || i == skip) continue;
            for (int p = b->rowptr[i] + 1; p < b->rowptr[i + 1]; ++p) {
                const int u = find(b->colidx[b->rowptr[i]]), v = find(b->colidx[p]);
                if (u != v) par[u] = v;
            }
        }
        std::vector<int> id(n, -1);
        ncomp = 0;
        for (int j = 0; j < n; ++j) {
            const int r = find(j);
            if (id[r] < 0) id[r] = ncomp++;
            comp_of_col[j] = id[r];
        }
        for (int i = 0; i < m; ++i) {
            if (coupling[i] || i == skip) { comp_of_row[i] = -1; continue; }
            if (b->rowptr[i + 1] == b->rowptr[i]) { comp_of_row[i] = ncomp++; continue; }   // empty row
            comp_of_row[i] = comp_of_col[b->colidx[b->rowptr[i]]];
        }
        ccols.assign(ncomp, 0);
        crows.assign(ncomp, 0);
        for (int j = 0; j < n; ++j) ccols[comp_of_col[j]]++;
        for (int i = 0; i < m; ++i)
            if (comp_of_row[i] >= 0) crows[comp_of_row[i]]++;
        // score: (oversized blocks, largest block) -- lower is better
        long over = 0, big = 0;
        for (int g = 0; g < ncomp; ++g) {
            over += (ccols[g] > CPL || crows[g] > RPL);
            big = std::max(big, (long)ccols[g] + crows[g]);
        }
        return over * 1000000L + big;
    };
    for (;;) {
        const long sc = blocks(-1);
        if (sc < 1000000L) break;                  // every block fits a lane
        if ((int)cpl.size() >= D) return 1;
        // next coupling row: the one whose removal leaves the fewest / smallest oversized blocks
        // (ties: the longer row)
        std::vector<int> cand;
        {
            std::vector<char> bad(ncomp, 0);
            for (int g = 0; g < ncomp; ++g) bad[g] = ccols[g] > CPL || crows[g] > RPL;
            for (int i = 0; i < m; ++i)
                if (!coupling[i] && comp_of_row[i] >= 0 && bad[comp_of_row[i]]) cand.push_back(i);
        }
        int best = -1, blen = -1;
        long bsc = 0;
        for (int i : cand) {
            const long s2 = blocks(i);
            const int len = b->rowptr[i + 1] - b->rowptr[i];
            if (best < 0 || s2 < bsc || (s2 == bsc && len > blen)) { best = i; bsc = s2; blen = len; }
        }
        if (best < 0) return 1;
        coupling[best] = 1;
        cpl.push_back(best);
    }
    // first-fit decreasing by (columns, rows)
    std::vector<int> order(ncomp);
    for (int g = 0; g < ncomp; ++g) order[g] = g;
    std::stable_sort(order.begin(), order.end(), [&](int u, int v) {
        return ccols[u] != ccols[v] ? ccols[u] > ccols[v] : crows[u] > crows[v];
    });
    std::vector<int> lane_c(LPS, 0), lane_r(LPS, 0), lane_of(ncomp, -1);
    for (int g : order) {
        int l = 0;
        while (l < LPS && (lane_c[l] + ccols[g] > CPL || lane_r[l] + crows[g] > RPL)) ++l;
        if (l == LPS) return 1;
        lane_of[g] = l;
        lane_c[l] += ccols[g];
        lane_r[l] += crows[g];
    }
    P.col_of.assign(LPS * CPL, -1);
    P.row_of.assign(LPS * RPL, -1);
    P.blk_p.assign(LPS * RPL * CPL, -1);
    P.cpl_row.assign(std::max(1, D), -1);
    P.cpl_p.assign(std::max(1, D * LPS * CPL), -1);
    std::vector<int> slot_of_col(n, -1), lane_of_col(n, -1);
    std::fill(lane_c.begin(), lane_c.end(), 0);
    std::fill(lane_r.begin(), lane_r.end(), 0);
    for (int j = 0; j < n; ++j) {
        const int l = lane_of[comp_of_col[j]];
        const int k = lane_c[l]++;
        P.col_of[l * CPL + k] = j;
        slot_of_col[j] = k;
        lane_of_col[j] = l;
    }
    for (int i = 0; i < m; ++i) {
        if (comp_of_row[i] < 0) continue;
        const int l = lane_of[comp_of_row[i]];
        const int r = lane_r[l]++;
        P.row_of[l * RPL + r] = i;
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) {
            const int j = b->colidx[p];
            if (lane_of_col[j] != l) return fail("plan_local: internal error (row split across lanes)");
            P.blk_p[(l * RPL + r) * CPL + slot_of_col[j]] = p;
        }
    }
    for (int d = 0; d < (int)cpl.size(); ++d) {
        const int i = cpl[d];
        P.cpl_row[d] = i;
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) {
            const int j = b->colidx[p];
            P.cpl_p[(d * LPS + lane_of_col[j]) * CPL + slot_of_col[j]] = p;
        }
    }
    return 0;
}

// Bound sides that are infinite in EVERY occupied slot of every scenario (the kernel drops their
// no-op clamps, pdhg_local.hip BI).  Columns that are nonants are excluded (fixing the nonants, the
// xhat evaluation, gives them finite boxes); rows can only gain infinite sides when fixed (row_bounds).
static unsigned long long local_inf_mask(const phg_batch* b, const LocalPlan& P, int LPS, int CPL, int RPL, int D) {
    std::vector<char> isn(b->n, 0);
    for (int k = 0; k < b->N; ++k) isn[b->nonant_col[k]] = 1;
    auto all_inf = [&](const double* v, int stride, int idx) {
        for (int s = 0; s < b->S; ++s)
            if (std::fabs(v[(size_t)s * stride + idx]) < 1e300) return false;
        return true;
    };
    unsigned long long m = 0;
    for (int k = 0; k < CPL && k < 16; ++k) {
        bool lo = true, hi = true, any = false;
        for (int l = 0; l < LPS; ++l) {
            const int j = P.col_of[l * CPL + k];
            if (j < 0) continue;
            any = true;
            if (isn[j]) { lo = hi = false; break; }
            lo = lo && all_inf(b->col_lo, b->n, j);
            hi = hi && all_inf(b->col_hi, b->n, j);
        }
        if (any && lo) m |= 1ull << k;
        if (any && hi) m |= 1ull << (16 + k);
    }
    for (int r = 0; r < RPL && r < 8; ++r) {
        bool lo = true, hi = true, any = false;
        for (int l = 0; l < LPS; ++l) {
            const int i = P.row_of[l * RPL + r];
            if (i < 0) continue;
            any = true;
            lo = lo && all_inf(b->row_lo, b->m, i);
            hi = hi && all_inf(b->row_hi, b->m, i);
        }
        if (any && lo) m |= 1ull << (32 + r);
        if (any && hi) m |= 1ull << (40 + r);
    }
    for (int d = 0; d < D && d < 4; ++d) {
        const int i = P.cpl_row[d];
        if (i < 0) continue;
        if (all_inf(b->row_lo, b->m, i)) m |= 1ull << (48 + d);
        if (all_inf(b->row_hi, b->m, i)) m |= 1ull << (52 + d);
    }
    return m;
}

// Bound sides that are FINITE in every occupied slot of every scenario (the kernel's restart /
// termination check then tests them at compile time, pdhg_local.hip BF).  Fixing the nonants keeps a
// finite column side finite (fixed_box); a row all of whose columns are nonants becomes free when
// they are fixed (row_bounds), so such rows never count as finite here.  Same bit layout as BI.
// nonant_fix false: the mask for solves that never fix the nonants (rows of nonants only may then
// count as finite: phg_handle::local_variant_free)
static unsigned long long local_fin_mask(const phg_batch* b, const LocalPlan& P, int LPS, int CPL, int RPL, int D,
                                         bool nonant_fix = true) {
    std::vector<char> isn(b->n, 0);
    for (int k = 0; k < b->N; ++k) isn[b->nonant_col[k]] = 1;
    auto all_fin = [&](const double* v, int stride, int idx) {
        for (int s = 0; s < b->S; ++s)
            if (!(std::fabs(v[(size_t)s * stride + idx]) < 1e300)) return false;
        return true;
    };
    auto fixable = [&](int i) {   // every column of row i a nonant
        if (!nonant_fix) return false;
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
            if (!isn[b->colidx[p]]) return false;
        return b->rowptr[i + 1] > b->rowptr[i];
    };
    unsigned long long m = 0;
    for (int k = 0; k < CPL && k < 16; ++k) {
        bool lo = true, hi = true, any = false;
        for (int l = 0; l < LPS; ++l) {
            const int j = P.col_of[l * CPL + k];
            if (j < 0) continue;
            any = true;
            lo = lo && all_fin(b->col_lo, b->n, j);
            hi = hi && all_fin(b->col_hi, b->n, j);
        }
        if (any && lo) m |= 1ull << k;
        if (any && hi) m |= 1ull << (16 + k);
    }
    for (int r = 0; r < RPL && r < 8; ++r) {
        bool lo = true, hi = true, any = false;
        for (int l = 0; l < LPS; ++l) {
            const int i = P.row_of[l * RPL + r];
            if (i < 0) continue;
            any = true;
            const bool fx = fixable(i);
            lo = lo && !fx && all_fin(b->row_lo, b->m, i);
            hi = hi && !fx && all_fin(b->row_hi, b->m, i);
        }
        if (any && lo) m |= 1ull << (32 + r);
        if (any && hi) m |= 1ull << (40 + r);
    }
    for (int d = 0; d < D && d < 4; ++d) {
        const int i = P.cpl_row[d];
        if (i < 0 || fixable(i)) continue;
        if (all_fin(b->row_lo, b->m, i)) m |= 1ull << (48 + d);
        if (all_fin(b->row_hi, b->m, i)) m |= 1ull << (52 + d);
    }
    return m;
}

// column slots holding a nonant in some lane (pdhg_local.hip QM: only they can carry a quadratic term)
static unsigned local_quad_mask(const phg_batch* b, const LocalPlan& P, int LPS, int CPL) {
    std::vector<char> isn(b->n, 0);
    for (int k = 0; k < b->N; ++k) isn[b->nonant_col[k]] = 1;
    unsigned m = 0;
    for (int l = 0; l < LPS; ++l)
        for (int k = 0; k < CPL && k < 32; ++k) {
            const int j = P.col_of[l * CPL + k];
            if (j >= 0 && isn[j]) m |= 1u << k;
        }
    return m;
}

static void local_slot_masks(const LocalPlan& plan, const int* sh, unsigned* mb, unsigned* mc) {
    const int LPS = sh[0], CPL = sh[1], RPL = sh[2], D = sh[3];
    *mb = *mc = 0;
    for (int l = 0; l < LPS; ++l) {
        for (int rr = 0; rr < RPL; ++rr)
            for (int k = 0; k < CPL; ++k)
                if (plan.blk_p[(l * RPL + rr) * CPL + k] >= 0) *mb |= 1u << (rr * CPL + k);
        for (int d = 0; d < D; ++d)
            for (int k = 0; k < CPL; ++k)
                if (plan.cpl_p[(d * LPS + l) * CPL + k] >= 0) *mc |= 1u << (d * CPL + k);
    }
}

// Shapes the default policy may take.  The all-coupling shape (one column per lane, up to 10
// replicated coupling rows: hydro) is correct but measured 3x slower than the wave-gather kernel on
// hydro 500-4 000 (0.966 vs 0.316 ms per PH iteration at 2 000: every row an all-reduce over 16 lanes
// each iteration, and twice the gather kernel's slowest solve; profiles/r06/hydro_layouts.json), so
// only an explicit PHG_LAYOUT_LOCAL gets it.
static bool local_shape_default(const int* sh) { return sh[3] <= 2; }

static int pick_local_variant(const phg_batch* b, LocalPlan& plan, int* sh) {
    for (int v = 0; v < pdhg_local_num_variants(); ++v) {
        pdhg_local_variant_shape(v, sh);
        if (!local_shape_default(sh)) continue;
        const int r = plan_local(b, sh[0], sh[1], sh[2], sh[3], plan);
        if (r < 0) return -2;
        if (r == 0) return v;
    }
    return -1;
}

// the free-solve variant only where its lane image is the same (same slot masks): else the safe one
static int local_pick_free(int safe, int free_v) {
    return pdhg_local_image_items(free_v) == pdhg_local_image_items(safe) ? free_v : safe;
}

static int build_local_layout(phg_handle* h, const phg_batch* b, bool any_shape) {
    int sh[4];
    LocalPlan plan;
    for (int v = 0; v < pdhg_local_num_variants(); ++v) {
        pdhg_local_variant_shape(v, sh);
        if (!any_shape && !local_shape_default(sh)) continue;
        const int r = plan_local(b, sh[0], sh[1], sh[2], sh[3], plan);
        if (r < 0) return -1;
        if (r > 0) continue;
        // slots occupied in at least one lane -> the pattern-specialised kernel of this shape
        const int LPS = sh[0], CPL = sh[1], RPL = sh[2], D = sh[3];
        unsigned mb = 0, mc = 0;
        local_slot_masks(plan, sh, &mb, &mc);
        // PHG_LOCAL_GENERIC=1 keeps the generic kernel (A/B of the specialisation)
        const char* gen = std::getenv("PHG_LOCAL_GENERIC");
        const unsigned long long bi = local_inf_mask(b, plan, LPS, CPL, RPL, D);
        const unsigned long long bf = local_fin_mask(b, plan, LPS, CPL, RPL, D);
        const unsigned qm = local_quad_mask(b, plan, LPS, CPL);
        h->local_variant = (gen && std::atoi(gen)) ? v : pdhg_local_pick_masked(v, mb, mc, bi, bf, qm);
        h->local_variant_free = local_pick_free(h->local_variant, (gen && std::atoi(gen)) ? v :
            pdhg_local_pick_masked(v, mb, mc, bi, local_fin_mask(b, plan, LPS, CPL, RPL, D, false), qm));
        h->local_shape_v = v;
        h->lp_col_of = plan.col_of;
        h->lp_row_of = plan.row_of;
        h->lp_cpl_row = plan.cpl_row;
        h->local_masks[0] = mb;
        h->local_masks[1] = mc;
        std::memcpy(h->lshape, sh, sizeof sh);
        int* p;
        if (dput(h, &p, plan.col_of.data(), plan.col_of.size())) return -1; h->loc.col_of = p;
        if (dput(h, &p, plan.row_of.data(), plan.row_of.size())) return -1; h->loc.row_of = p;
        if (dput(h, &p, plan.blk_p.data(), plan.blk_p.size())) return -1; h->loc.blk_p = p;
        if (dput(h, &p, plan.cpl_row.data(), plan.cpl_row.size())) return -1; h->loc.cpl_row = p;
        if (dput(h, &p, plan.cpl_p.data(), plan.cpl_p.size())) return -1; h->loc.cpl_p = p;
        {   // nonant index of every column slot (the prologue's W / rho / xbar reads)
            std::vector<int> col_nonant(b->n, -1), kk(plan.col_of.size(), -1);
            for (int q = 0; q < b->N; ++q) col_nonant[b->nonant_col[q]] = q;
            for (size_t e = 0; e < kk.size(); ++e)
                if (plan.col_of[e] >= 0) kk[e] = col_nonant[plan.col_of[e]];
            if (dput(h, &p, kk.data(), kk.size())) return -1; h->loc.slot_kk = p;
        }
        return 0;
    }
    g_err = "phg_load_batch: the pattern has no lane-local layout (blocks too large or too many coupling rows)";
    return 1;
}

static int build_ph_tables(phg_handle* h, const phg_batch* b) {
    const int S = b->S, N = b->N, L = b->L;
    // level offsets: nonants must be grouped by level in node-list order
    std::vector<int> level_kofs(L, -1);
    for (int k = 0; k < N; ++k) {
        const int lv = b->nonant_level[k];
        if (lv < 0 || lv >= L) return fail("phg_load_batch: nonant_level out of range");
        if (level_kofs[lv] < 0) level_kofs[lv] = k;
        if (k > 0 && b->nonant_level[k] < b->nonant_level[k - 1])
            return fail("phg_load_batch: nonants must be ordered by tree level");
        if (b->nonant_pos[k] != k - level_kofs[lv]) return fail("phg_load_batch: nonant_pos mismatch");
    }
    int maxk = 1;
    for (int lv = 0; lv < L; ++lv) maxk = std::max(maxk, b->level_len[lv]);
    std::vector<int> node_level(b->n_nodes, -1);
    for (int s = 0; s < S; ++s)
        for (int lv = 0; lv < L; ++lv) {
            const int g = b->scen_node[s * L + lv];
            if (g < 0 || g >= b->n_nodes) return fail("phg_load_batch: scen_node out of range");
            node_level[g] = lv;
        }
    for (int g = 1; g < b->n_nodes; ++g)
        if (b->node_off[g] < b->node_off[g - 1]) return fail("phg_load_batch: node_off must increase");
    // node segments: contiguous scenario ranges per node, chunked
    std::vector<std::vector<NodeSeg>> per_node(b->n_nodes);
    // segments per level cap (PHG_NODESEG_MAX: tuning knob for tools/ph_update_sweep.py)
    int seg_max = 256;   // (512 -> 256 measured: S*N 1e6 / 1e7 / 1e8 33 -> 29, 73 -> 71, ~670 -> ~657 us)
    if (const char* ev = std::getenv("PHG_NODESEG_MAX")) seg_max = std::max(1, std::atoi(ev));
    const bool seg_env = std::getenv("PHG_NODESEG_MAX") != nullptr;
    for (int lv = 0; lv < L; ++lv) {
        const int klen = b->level_len[lv];
        // narrow levels get more segments: a node-sum workgroup covers 256 nonants of its segment
        // (blockIdx.y), so with klen <= 256 the grid is the segment count alone -- 1024 of them keep
        // ~4 workgroups per CU in flight (S N = 1e8 as 1e6 x 100: 256 segments ran at 2.3 TB/s)
        const int seg_cap = seg_env ? seg_max : std::max(seg_max, 1024 / std::max(1, (klen + 255) / 256));
        // ~8 scenarios per thread of a 256-thread workgroup: enough workgroups to hide the load
        // latency at small S, whole-row coalesced streaming at large S
        // and at most ~256 segments per level, so the final per-node sums stay short at large S
        const int chunk = std::max(klen >= 256 ? 8 : 8 * (256 / std::max(1, klen)), (S + seg_cap - 1) / seg_cap);
        int s = 0;
        while (s < S) {
            const int g = b->scen_node[s * L + lv];
            if (!per_node[g].empty() && per_node[g].back().s1 != s)
                return fail("phg_load_batch: scenarios of a tree node must be contiguous");
            int e = s;
            while (e < S && b->scen_node[e * L + lv] == g && e - s < chunk) ++e;
            per_node[g].push_back(NodeSeg{lv, g, s, e, level_kofs[lv], klen, 0});
            s = e;
        }
    }
    std::vector<NodeSeg> segs;
    std::vector<int> first(b->n_nodes + 1, 0);
    for (int g = 0; g < b->n_nodes; ++g) {
        first[g] = (int)segs.size();
        for (auto& sg : per_node[g]) segs.push_back(sg);
    }
    first[b->n_nodes] = (int)segs.size();
    // conv segments: virtual-rank slices of the global scenario list (sputils.py:819-826)
    const int P = std::max(1, b->virt_nproc);
    const int Sg = b->S_global > 0 ? b->S_global : S;
    std::vector<int> vr(S, 0);
    if (P > 1) {
        const double avg = (double)Sg / (double)P;
        for (int s = 0; s < S; ++s) {
            const int gs = b->scen_global0 + s;
            int v = 0;
            while (v + 1 < P && gs >= (int)((v + 1) * avg)) ++v;
            vr[s] = v;
        }
    }
    std::vector<int> cv, cs0, cs1, vfirst(P + 1, 0);
    // ~8 elements per thread, at most ~1024 segments
    const int cchunk = std::max(std::max(1, 2048 / std::max(1, N)), (S + 1023) / 1024);
    {
        int s = 0;
        std::vector<std::vector<int>> tmp0(P), tmp1(P);
        while (s < S) {
            const int v = vr[s];
            int e = s;
            while (e < S && vr[e] == v && e - s < cchunk) ++e;
            tmp0[v].push_back(s);
            tmp1[v].push_back(e);
            s = e;
        }
        for (int v = 0; v < P; ++v) {
            vfirst[v] = (int)cv.size();
            for (size_t i = 0; i < tmp0[v].size(); ++i) {
                cv.push_back(v);
                cs0.push_back(tmp0[v][i]);
                cs1.push_back(tmp1[v][i]);
            }
        }
        vfirst[P] = (int)cv.size();
    }
    // xbar slot of (s, k)
    std::vector<int> xidx((size_t)S * N);
    for (int s = 0; s < S; ++s)
        for (int k = 0; k < N; ++k)
            xidx[(size_t)s * N + k] = b->node_off[b->scen_node[s * L + b->nonant_level[k]]] + b->nonant_pos[k];
    bool root_only = true;   // x-bar slot == k for every scenario (two-stage): w_update_kernel<true>
    for (size_t e = 0; e < xidx.size() && root_only; ++e) root_only = xidx[e] == (int)(e % (size_t)N);
    PhArgs& a = h->ph;
    a.rho_k = nullptr;   // until phg_set(PHG_F_RHO) finds rho the same in every scenario
    a.root_only = root_only ? 1 : 0;
    a.S = S; a.N = N; a.N_tot = b->N_tot; a.L = L; a.P = P; a.maxk = maxk; a.n_nodes = b->n_nodes;
    a.n_seg = (int)segs.size();
    a.n_cseg = (int)cv.size();
    {   // final node-sum reduction: ~2K partial loads per workgroup, at most 128 workgroups (far
        // below the resident capacity, so the ranked workgroups' spin never starves a late one)
        long loads = 0;
        for (int g = 0; g < b->n_nodes; ++g)   // nodes without local scenarios have no segments
            if (node_level[g] >= 0) loads += 2L * (first[g + 1] - first[g]) * b->level_len[node_level[g]];
        // PHG_NFINAL_LOADS: partial loads per final workgroup (tuning knob; 1 024 from 2 048 in round
        // 6: farmer 10 000's node-sum head 12.5 vs 13.3 us, K = 10 vs 5 ranks; 1 250 unchanged)
        long per = 1024;
        if (const char* ev = std::getenv("PHG_NFINAL_LOADS")) per = std::max(1L, std::atol(ev));
        a.n_final = (int)std::min<long>(128, std::max<long>(1, (loads + per - 1) / per));
    }
    {
        NodeSeg* p;
        if (dput(h, &p, segs.data(), segs.size())) return -1;
        a.seg = p;
    }
    {   // the solve tail's tables (ph_tail.h): every scenario's node segment per level and conv
        // segment, the unit counters, and the final reduction's slot plan -- node_sum_final's ranks
        // (K = the node-sum grid's min(n_final, workgroups)), each element's T strided sums in T
        // aligned slots, elements packed widest T first so every run stays T-aligned
        std::vector<int> sseg((size_t)S * L, 0), scs(S, 0);
        for (int g = 0; g < (int)segs.size(); ++g)
            for (int s2 = segs[g].s0; s2 < segs[g].s1; ++s2) sseg[(size_t)s2 * L + segs[g].level] = g;
        for (size_t c = 0; c < cs0.size(); ++c)
            for (int s2 = cs0[c]; s2 < cs1[c]; ++s2) scs[s2] = (int)c;
        const long ny = (maxk + 255) / 256;
        const int K = (int)std::min<long>(a.n_final, (long)segs.size() * ny);
        struct El { int e, T, g0, cnt, i; };
        std::vector<El> els;
        for (int r = 0; r < K; ++r) {
            const int e_lo = (int)((long)b->N_tot * r / K), e_hi = (int)((long)b->N_tot * (r + 1) / K);
            const int ne = e_hi - e_lo;
            int T = 1;
            while (T < 64 && T * 2 * ne <= 256) T *= 2;
            for (int e = e_lo; e < e_hi; ++e) {
                int lo = 0, hi = b->n_nodes - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (b->node_off[mid] <= e) lo = mid; else hi = mid - 1;
                }
                els.push_back({e, T, first[lo], first[lo + 1] - first[lo], e - b->node_off[lo]});
            }
        }
        std::stable_sort(els.begin(), els.end(), [](const El& x, const El& y) { return x.T > y.T; });
        // slot = int4 {element, first segment, terms | stride << 16, position in the node}
        std::vector<int> fin;
        for (const El& el : els)
            for (int sub = 0; sub < el.T; ++sub) {
                const int J = sub < el.cnt ? (el.cnt - sub + el.T - 1) / el.T : 0;
                fin.insert(fin.end(), {el.e, el.g0 + sub, J | (el.T << 16), el.i});
            }
        while ((fin.size() / 4) % 64) fin.insert(fin.end(), {-1, 0, 1 << 16, 0});
        h->tail_nfin = (int)(fin.size() / 4);
        if (dput(h, &h->tail_scen_seg, sseg.data(), sseg.size())) return -1;
        if (dput(h, &h->tail_scen_cseg, scs.data(), scs.size())) return -1;
        if (dput(h, &h->tail_fin, fin.data(), fin.size())) return -1;
        if (dalloc(h, &h->tail_segcnt, segs.size())) return -1;
        if (dalloc(h, &h->tail_csegcnt, cs0.size())) return -1;
        if (dalloc(h, &h->tail_done, 1)) return -1;
    }
    int* ip;
    double* dp;
    if (dalloc(h, &dp, (size_t)segs.size() * 2 * maxk)) return -1; a.segpart = dp;
    if (dput(h, &ip, first.data(), first.size())) return -1; a.node_first_seg = ip;
    if (dput(h, &ip, b->node_off, b->n_nodes)) return -1; a.node_off = ip;
    if (dput(h, &ip, node_level.data(), node_level.size())) return -1; a.node_level = ip;
    if (dput(h, &ip, b->level_len, L)) return -1; a.level_len = ip;
    if (dput(h, &ip, level_kofs.data(), L)) return -1; a.level_kofs = ip;
    if (dput(h, &ip, b->nonant_level, N)) return -1; a.nonant_level = ip;
    if (dput(h, &dp, b->prob_coeff, (size_t)S * L)) return -1; a.pc = dp;
    a.pcv = nullptr;
    if (b->prob_coeff_var) {
        if (dput(h, &dp, b->prob_coeff_var, (size_t)S * N)) return -1;
        a.pcv = dp;
    }
    if (dput(h, &ip, cv.data(), cv.size())) return -1; a.cseg_v = ip;
    if (dput(h, &ip, cs0.data(), cs0.size())) return -1; a.cseg_s0 = ip;
    if (dput(h, &ip, cs1.data(), cs1.size())) return -1; a.cseg_s1 = ip;
    if (dalloc(h, &dp, cv.size())) return -1; a.csegpart = dp;
    if (dalloc(h, &ip, 2 * cv.size())) return -1; a.csegbad = ip;
    {
        unsigned* t;
        if (dalloc(h, &t, 3)) return -1;
        a.ticket = t;
        if (dalloc(h, &t, 4)) return -1;
        a.fticket = t;
    }
    if (dput(h, &ip, vfirst.data(), vfirst.size())) return -1; a.vr_first = ip;
    if (dput(h, &ip, xidx.data(), xidx.size())) return -1; h->xidx = ip;
    a.xidx = h->xidx;
    if (dalloc(h, &h->conv_s, (size_t)S)) return -1;
    if (dalloc(h, &h->fold_st, (size_t)S)) return -1;
    a.conv_s = h->conv_s;      // the folded update's per-scenario partials (fold_conv_kernel, node sums)
    a.fold_st = h->fold_st;
    a.fold_conv = 0;
    if (dalloc(h, &h->packed, 2 * (size_t)b->N_tot + 2 * (size_t)P + 3)) return -1;
    h->nodesum = h->packed;
    h->convpart = h->packed + 2 * (size_t)b->N_tot;
    if (dalloc(h, &h->gate, 4)) return -1;
    CK(hipHostMalloc((void**)&h->gate_host, 8 * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
    for (int i = 0; i < 8; ++i) h->gate_host[i] = 0.0;
    return 0;
}

// Workgroup-per-scenario layout (pdhg_block.hip): owner slots and <= kPiece-entry pieces.
// Returns 0 (built), 1 (no variant fits), -1 (error).  Values are gathered into the piece layout
// after preconditioning (build_block_values).
static constexpr int kPiece = 8;

static int build_block_layout(phg_handle* h, const phg_batch* b, const std::vector<int>& colptr,
                              const std::vector<int>& csc_row, const std::vector<int>& csc_p, bool want_delta) {
    const int n = b->n, m = b->m;
    // pieces in row (column) order
    std::vector<int> rpf(m), rpc(m), cpf(n), cpc(n);
    std::vector<int> rps, rpl, cps, cpl;   // start position, length
    for (int i = 0; i < m; ++i) {
        rpf[i] = (int)rps.size();
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; p += kPiece) {
            rps.push_back(p);
            rpl.push_back(std::min(kPiece, b->rowptr[i + 1] - p));
        }
        rpc[i] = (int)rps.size() - rpf[i];
    }
    for (int j = 0; j < n; ++j) {
        cpf[j] = (int)cps.size();
        for (int e = colptr[j]; e < colptr[j + 1]; e += kPiece) {
            cps.push_back(e);
            cpl.push_back(std::min(kPiece, colptr[j + 1] - e));
        }
        cpc[j] = (int)cps.size() - cpf[j];
    }
    const int n_pad = (n + 1) & ~1, m_pad = (m + 1) & ~1;
    const int rlen = rpl.empty() ? 0 : *std::max_element(rpl.begin(), rpl.end());
    const int clen = cpl.empty() ? 0 : *std::max_element(cpl.begin(), cpl.end());
    // PHG_BLOCK_STREAM=1: skip the register-resident variants (A/B of the two forms)
    const char* es = std::getenv("PHG_BLOCK_STREAM");
    const bool stream_only = es && std::atoi(es) != 0;
    // every column one piece (then piece j is column j, in the column owner's thread and slot)
    bool col_one_piece = true;
    for (int j = 0; j < n && col_one_piece; ++j) col_one_piece = cpf[j] == j && cpc[j] == 1;
    // PHG_BLOCK_CL=0: skip the column-local variants (A/B)
    const char* ec = std::getenv("PHG_BLOCK_CL");
    const bool cl_off = ec && std::atoi(ec) == 0;
    // the variants whose row piece sums issue their loads together (sslp 4 096: 8.20 vs 8.86 ms per PH
    // iteration, the same bits); PHG_PSUM=0 skips them (A/B)
    const char* eps_ = std::getenv("PHG_PSUM");
    const bool psum = !(eps_ && std::atoi(eps_) == 0);
    // row segments (SEG variants): every row's pieces in an aligned 1 / 2 / 4 / 8 / 16-lane segment of
    // one row slot, rows placed longest segment first, a slot filled before the next (which keeps
    // every segment aligned); seg_len[i], seg_pos[i] = slot * NT + lane.  Returns the slots used
    // (NT lanes each), or a large number when a row does not fit.
    const char* esg = std::getenv("PHG_BLOCK_SEG");
    const bool seg_off = esg && std::atoi(esg) == 0;
    std::vector<int> seg_len(m), seg_pos(m);
    auto seg_plan = [&](int NT_, int maxlen) {
        for (int i = 0; i < m; ++i) {
            const int c = rpc[i];
            if (c > maxlen) return 1 << 20;
            seg_len[i] = c <= 1 ? 1 : (c <= 2 ? 2 : (c <= 4 ? 4 : (c <= 8 ? 8 : 16)));
        }
        std::vector<int> ord(m);
        for (int i = 0; i < m; ++i) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](int u, int v) { return seg_len[u] > seg_len[v]; });
        int slot = 0, lane = 0;
        for (int i : ord) {
            if (lane + seg_len[i] > NT_) { ++slot; lane = 0; }
            seg_pos[i] = slot * NT_ + lane;
            lane += seg_len[i];
        }
        return m > 0 ? slot + 1 : 1 << 20;
    };
    // PHG_BLOCK_MINNT: skip the variants with fewer threads (A/B of the workgroup size)
    const char* emn = std::getenv("PHG_BLOCK_MINNT");
    const int min_nt = emn ? std::atoi(emn) : 0;
    int sh[12], chosen = -1;
    for (int v = 0; v < pdhg_block_num_variants(); ++v) {
        pdhg_block_variant_shape(v, sh);
        if (sh[10]) continue;   // unit twins: chosen by build_block_values
        if (sh[0] < min_nt) continue;
        if (sh[11] && (seg_off || seg_plan(sh[0], sh[11] / 1) > sh[2])) continue;
        if ((sh[9] != 0) != psum && sh[9] != 0) continue;
        const int NT = sh[0], CPL = sh[1], RPL = sh[2], PPT = sh[3], QPT = sh[4], RE = sh[5], CE = sh[6], CL = sh[7];
        if ((sh[8] != 0) != want_delta) continue;   // delta form: the on-the-fly scaling variants
        if (n > CPL * NT || m > RPL * NT || (!sh[11] && (int)rps.size() > PPT * NT) || (int)cps.size() > QPT * NT) continue;
        if (RE > 0 && (stream_only || rlen > RE || clen > CE)) continue;   // pieces must fit the registers
        if (CL && (!col_one_piece || cl_off)) continue;
        if (pdhg_block_lds_bytes(v, n_pad, m_pad, 0, 0) > 160 * 1024) continue;
        chosen = v;
        break;
    }
    if (chosen < 0) {
        char msg[256];
        snprintf(msg, sizeof msg, "phg_load_batch: no workgroup PDHG variant fits n=%d m=%d (%zu/%zu pieces)", n, m,
                 rps.size(), cps.size());
        g_err = msg;
        return 1;
    }
    pdhg_block_variant_shape(chosen, sh);
    const int NT = sh[0], CPL = sh[1], RPL = sh[2], PPT = sh[3], QPT = sh[4];
    h->block_variant = chosen;
    std::memcpy(h->bshape, sh, sizeof sh);
    BlockLayout& L = h->blk;
    L.n_pad = n_pad;
    L.m_pad = m_pad;
    std::vector<int> col_of(CPL * NT, -1), colf(CPL * NT, 0), colc(CPL * NT, 0);
    for (int j = 0; j < n; ++j) {
        const int idx = (j / NT) * NT + j % NT;
        col_of[idx] = j; colf[idx] = cpf[j]; colc[idx] = cpc[j];
    }
    std::vector<int> row_of(RPL * NT, -1), rowf(RPL * NT, 0), rowc(RPL * NT, 0);
    if (sh[11]) {
        // row segments: the row's owner is its segment's first lane (row_pcnt = segment length), its
        // pieces the segment's lanes of the same slot; the piece list in slot-lane order, empty
        // pieces on the padding lanes
        seg_plan(NT, sh[11]);
        std::vector<int> lps((size_t)RPL * NT, 0), lpl((size_t)RPL * NT, 0);
        for (int i = 0; i < m; ++i) {
            const int l0 = seg_pos[i];
            row_of[l0] = i; rowf[l0] = l0; rowc[l0] = seg_len[i];
            for (int q = 0; q < rpc[i]; ++q) { lps[l0 + q] = rps[rpf[i] + q]; lpl[l0 + q] = rpl[rpf[i] + q]; }
        }
        rps.swap(lps);
        rpl.swap(lpl);
    } else {
        for (int i = 0; i < m; ++i) {
            const int idx = (i / NT) * NT + i % NT;
            row_of[idx] = i; rowf[idx] = rpf[i]; rowc[idx] = rpc[i];
        }
    }
    // piece-major entry layout
    auto lay = [&](const std::vector<int>& ps, const std::vector<int>& pl, int SLOTS, int* kk,
                   const std::function<int(int)>& idx_of, const std::function<int(int)>& pos_of,
                   std::vector<int>& idx, std::vector<int>& perm) {
        for (int sl = 0; sl < 8; ++sl) kk[sl] = 0;
        for (size_t p = 0; p < ps.size(); ++p) kk[p / NT] = std::max(kk[p / NT], pl[p]);
        int tot = 0;
        std::vector<int> off(SLOTS + 1, 0);
        for (int sl = 0; sl < SLOTS; ++sl) { off[sl] = tot; tot += kk[sl] * NT; }
        idx.assign(std::max(1, tot), 0);
        perm.assign(std::max(1, tot), -1);
        for (size_t p = 0; p < ps.size(); ++p) {
            const int sl = (int)p / NT, t = (int)p % NT;
            for (int k = 0; k < pl[p]; ++k) {
                const int e = off[sl] + k * NT + t;
                idx[e] = idx_of(ps[p] + k);
                perm[e] = pos_of(ps[p] + k);
            }
        }
        return tot;
    };
    std::vector<int> ridx, cidx;
    const int rtot = lay(rps, rpl, PPT, L.rk, [&](int p) { return b->colidx[p]; }, [&](int p) { return p; }, ridx,
                         h->block_rperm);
    const int ctot = lay(cps, cpl, QPT, L.ck, [&](int e) { return csc_row[e]; }, [&](int e) { return csc_p[e]; }, cidx,
                         h->block_cperm);
    (void)rtot; (void)ctot;
    int* p;
    if (dput(h, &p, col_of.data(), col_of.size())) return -1; L.col_of = p;
    if (dput(h, &p, colf.data(), colf.size())) return -1; L.col_pfirst = p;
    if (dput(h, &p, colc.data(), colc.size())) return -1; L.col_pcnt = p;
    if (dput(h, &p, row_of.data(), row_of.size())) return -1; L.row_of = p;
    if (dput(h, &p, rowf.data(), rowf.size())) return -1; L.row_pfirst = p;
    if (dput(h, &p, rowc.data(), rowc.size())) return -1; L.row_pcnt = p;
    if (dput(h, &p, ridx.data(), ridx.size())) return -1; L.ridx = p;
    if (dput(h, &p, cidx.data(), cidx.size())) return -1; L.cidx = p;
    return 0;
}

// One-wave-per-scenario layout (pdhg_wave.hip) for a matrix shared by every scenario: column order =
// the nonants first (their slots carry the prox diagonal), then the rest; every column's <= CE
// entries; rows and 8-entry row pieces dealt over the lanes.  Returns 0 (built), 1 (does not fit:
// the caller tries the workgroup layout), -1 (error).  PHG_WAVE=0: never (A/B runs).
static int build_wave_layout(phg_handle* h, const phg_batch* b, const std::vector<int>& colptr,
                             const std::vector<int>& csc_row, const std::vector<int>& csc_p) {
    const char* ew = std::getenv("PHG_WAVE");
    if ((ew && std::atoi(ew) == 0) || !h->vals_shared) return 1;
    const int n = b->n, m = b->m, N = b->N;
    int cmax = 0;
    for (int j = 0; j < n; ++j) cmax = std::max(cmax, colptr[j + 1] - colptr[j]);
    std::vector<int> rps, rpl, rpf(m), rpc(m);
    for (int i = 0; i < m; ++i) {
        rpf[i] = (int)rps.size();
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; p += 8) {
            rps.push_back(p);
            rpl.push_back(std::min(8, b->rowptr[i + 1] - p));
        }
        rpc[i] = (int)rps.size() - rpf[i];
    }
    int sh[6], chosen = -1;
    for (int v = 0; v < pdhg_wave_num_variants(); ++v) {
        pdhg_wave_variant_shape(v, sh);
        const int CPL = sh[0], RPL = sh[1], PPT = sh[2], CE = sh[3], NSL = sh[4];
        if (n > CPL * 64 || m > RPL * 64 || (int)rps.size() > PPT * 64 || cmax > CE || N > NSL * 64) continue;
        chosen = v;
        break;
    }
    if (chosen < 0) return 1;
    pdhg_wave_variant_shape(chosen, sh);
    const int CPL = sh[0], RPL = sh[1], PPT = sh[2], CE = sh[3];
    WaveLayout& L = h->wv;
    L.n_pad = CPL * 64;       // x by column position (empty positions stay 0)
    L.m_pad = (m + 1) & ~1;
    L.wave_doubles = L.n_pad + L.m_pad + PPT * 64;
    if (pdhg_wave_lds_bytes(chosen, L.wave_doubles) > 160 * 1024) return 1;
    h->wave_variant = chosen;
    std::memcpy(h->wshape, sh, sizeof sh);
    // column order: nonants first
    std::vector<int> order;
    std::vector<char> isn(n, 0);
    for (int k = 0; k < N; ++k) { order.push_back(b->nonant_col[k]); isn[b->nonant_col[k]] = 1; }
    for (int j = 0; j < n; ++j) if (!isn[j]) order.push_back(j);
    std::vector<int> col_of(CPL * 64, -1), cidx((size_t)CPL * 64 * CE, 0), pos(n, 0);
    h->wave_cperm.assign((size_t)CPL * 64 * CE, -1);
    for (int p = 0; p < n; ++p) {
        const int j = order[p], slot = p / 64, ln = p % 64;
        col_of[slot * 64 + ln] = j;
        pos[j] = p;
        for (int e = 0; e < colptr[j + 1] - colptr[j]; ++e) {
            const size_t q = ((size_t)slot * 64 + ln) * CE + e;
            cidx[q] = csc_row[colptr[j] + e];
            h->wave_cperm[q] = csc_p[colptr[j] + e];
        }
    }
    std::vector<int> row_of(RPL * 64, -1), rowf(RPL * 64, 0), rowc(RPL * 64, 0);
    for (int i = 0; i < m; ++i) { row_of[i] = i; rowf[i] = rpf[i]; rowc[i] = rpc[i]; }
    std::vector<int> ridx((size_t)PPT * 8 * 64, 0);
    h->wave_rperm.assign((size_t)PPT * 8 * 64, -1);
    for (size_t p = 0; p < rps.size(); ++p) {
        const int slot = (int)p / 64, ln = (int)p % 64;
        for (int e = 0; e < rpl[p]; ++e) {
            const size_t q = ((size_t)slot * 8 + e) * 64 + ln;
            ridx[q] = pos[b->colidx[rps[p] + e]];
            h->wave_rperm[q] = rps[p] + e;
        }
    }
    int* ip;
    if (dput(h, &ip, col_of.data(), col_of.size())) return -1; L.col_of = ip;
    if (dput(h, &ip, cidx.data(), cidx.size())) return -1; L.cidx = ip;
    if (dput(h, &ip, row_of.data(), row_of.size())) return -1; L.row_of = ip;
    if (dput(h, &ip, rowf.data(), rowf.size())) return -1; L.row_pfirst = ip;
    if (dput(h, &ip, rowc.data(), rowc.size())) return -1; L.row_pcnt = ip;
    if (dput(h, &ip, ridx.data(), ridx.size())) return -1; L.ridx = ip;
    return 0;
}

// the wave layout's value copies (scenario 0's scaled matrix = every scenario's)
static int build_wave_values(phg_handle* h) {
    WaveLayout& L = h->wv;
    int* rperm;
    int* cperm;
    double* rv;
    double* cv;
    const int Er = (int)h->wave_rperm.size(), Ec = (int)h->wave_cperm.size();
    if (dput(h, &rperm, h->wave_rperm.data(), Er)) return -1;
    if (dput(h, &cperm, h->wave_cperm.data(), Ec)) return -1;
    if (dalloc(h, &rv, Er)) return -1;
    if (dalloc(h, &cv, Ec)) return -1;
    CK(piece_gather_launch(h->vals, h->nnz, rperm, Er, 1, rv, h->stream));
    CK(piece_gather_launch(h->vals, h->nnz, cperm, Ec, 1, cv, h->stream));
    L.rvals = rv;
    L.cvals = cv;
    return 0;
}

// Unit form (BlockLayout::rcode): when every constant entry of the delta form is -1, 0 or +1 (network
// rows: netdes's flow balances and the y side of its capacity rows), the chosen variant's unit twin
// keeps the whole matrix in LDS as 16-bit entry codes plus the scenario's varying entry rows.  Needs
// the twin's LDS to fit and n, m < 32 767.  PHG_UNIT=0: never (A/B runs).
static int build_unit_codes(phg_handle* h, const double* rv, const double* cv) {
    BlockLayout& L = h->blk;
    const char* eu = std::getenv("PHG_UNIT");
    // codes are 16-bit LDS byte addresses: x, y and the zero slot after them must sit below 64 KiB
    if ((eu && std::atoi(eu) == 0) || (long)(L.n_pad + L.m_pad + 1) * 8 > 0xFFF8) return 0;
    int twin = -1, sh[12];
    for (int v = 0; v < pdhg_block_num_variants() && twin < 0; ++v) {
        pdhg_block_variant_shape(v, sh);
        if (sh[10] && std::equal(sh, sh + 10, h->bshape) && sh[11] == h->bshape[11]) twin = v;
    }
    if (twin < 0 || pdhg_block_lds_bytes(twin, L.n_pad, L.m_pad, L.nd_r + L.nd_c, L.er + L.ec) > 160 * 1024) return 0;
    const int NT = h->bshape[0];
    // entry code: the LDS byte address of the entry's x (row pieces: xl at 0) or y (column pieces: yl
    // at n_pad doubles) with the value's sign in bit 0; padding -> the zero slot after yl
    const unsigned zero_addr = (unsigned)(L.n_pad + L.m_pad) * 8u;
    auto codes = [&](const double* dv, const int* didx, int E, const int* drow, int base, std::vector<short>& out) {
        std::vector<double> val(E);
        std::vector<int> idx(E);
        if (hipMemcpy(val.data(), dv, (size_t)E * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(idx.data(), didx, (size_t)E * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        out.assign(std::max(1, E), 0);
        for (int e = 0; e < E; ++e) {
            const unsigned c = (unsigned)(base + idx[e]) * 8u;
            if (drow[e / NT] >= 0) { out[e] = (short)c; continue; }   // varying row: its value from rvd / cvd
            if (val[e] == 1.0) out[e] = (short)c;
            else if (val[e] == -1.0) out[e] = (short)(c | 1u);
            else if (val[e] == 0.0 && !std::signbit(val[e])) out[e] = (short)zero_addr;
            else return 1;   // a constant entry that is not a unit
        }
        return 0;
    };
    CK(hipStreamSynchronize(h->stream));   // the piece gathers wrote rv / cv
    std::vector<short> rc, cc;
    int r = codes(rv, L.ridx, L.er, L.rdrow, 0, rc);
    if (r == 0) r = codes(cv, L.cidx, L.ec, L.cdrow, L.n_pad, cc);
    if (r < 0) return fail("phg_load_batch: reading the piece values back failed");
    if (r > 0) return 0;
    short* p;
    if (dput(h, &p, rc.data(), rc.size())) return -1; L.rcode = p;
    if (dput(h, &p, cc.data(), cc.size())) return -1; L.ccode = p;
    h->block_variant = twin;
    pdhg_block_variant_shape(twin, h->bshape);
    return 0;
}

// Default primal-weight smoothing theta (omega <- r^theta omega^(1 - theta) at a restart, r the
// restart's ||dy|| / ||dx||) by subproblem size, measured per PH iteration on MI355X (DESIGN.md,
// round 3): farmer (n 120) 0.8 best (0.5: -2 %, 0.3: -12 %); sslp (705) 0.6-0.8; hydro 0.6 by 4 %;
// netdes (2 940) 0.5 by 8-11 %; UC (20 400) 0.05: 83 vs 641 ms per PH iteration (PH iterations
// 1-8 at 64 scenarios; mean PDHG iterations per solve 930 vs 13 609, the slowest 12 892 vs 58 968).
// PHG_THETA overrides it (A/B runs).
static double theta_default(int n) {
    static const double env = [] {
        const char* e = std::getenv("PHG_THETA");
        const double v = e ? std::atof(e) : 0.0;
        return v > 0.0 && v <= 1.0 ? v : 0.0;
    }();
    if (env > 0.0) return env;
    return n >= 10000 ? 0.05 : (n >= 2000 ? 0.5 : 0.8);
}

// piece-major copies of the (preconditioned) values; one copy when every scenario has the same A
static int build_block_values(phg_handle* h, const double* raw) {
    BlockLayout& L = h->blk;
    L.vscale = h->delta_scale ? 1 : 0;
    const double* src = h->delta_scale ? raw : h->vals;   // unscaled values for the delta form
    const int Er = (int)h->block_rperm.size(), Ec = (int)h->block_cperm.size();
    const bool one = h->vals_shared || h->delta_scale;   // one copy of the (constant) entries
    const int Sv = one ? 1 : h->S;
    const int NT = h->bshape[0];
    int* rperm;
    int* cperm;
    double* rv;
    double* cv;
    if (dput(h, &rperm, h->block_rperm.data(), Er)) return -1;
    if (dput(h, &cperm, h->block_cperm.data(), Ec)) return -1;
    if (dalloc(h, &rv, (size_t)Sv * Er)) return -1;
    if (dalloc(h, &cv, (size_t)Sv * Ec)) return -1;
    CK(piece_gather_launch(src, h->nnz, rperm, Er, Sv, rv, h->stream));
    CK(piece_gather_launch(src, h->nnz, cperm, Ec, Sv, cv, h->stream));
    L.rvals = rv;
    L.cvals = cv;
    L.vstride_r = one ? 0 : Er;
    L.vstride_c = one ? 0 : Ec;
    // delta form: per-scenario copies of the entry rows that hold a varying entry
    auto deltas = [&](const std::vector<int>& perm, int E, int* drow, const double** dv, long* dstride) {
        for (int R = 0; R < 32; ++R) drow[R] = -1;
        *dv = nullptr;
        *dstride = 0;
        if (!h->delta_scale) return 0;
        const int rows = E / NT;
        if (rows > 32) return fail("phg_load_batch: piece layout has more than 32 entry rows");
        std::vector<int> dperm;
        int nd = 0;
        for (int R = 0; R < rows; ++R) {
            bool any = false;
            for (int t = 0; t < NT; ++t) {
                const int p = perm[(size_t)R * NT + t];
                any |= p >= 0 && h->vary[p];
            }
            if (!any) continue;
            drow[R] = nd++;
            dperm.insert(dperm.end(), perm.begin() + (size_t)R * NT, perm.begin() + (size_t)(R + 1) * NT);
        }
        if (!nd) return 0;
        int* dp;
        double* out;
        if (dput(h, &dp, dperm.data(), dperm.size())) return -1;
        if (dalloc(h, &out, (size_t)h->S * dperm.size())) return -1;
        CK(piece_gather_launch(src, h->nnz, dp, (int)dperm.size(), h->S, out, h->stream));
        *dv = out;
        *dstride = (long)dperm.size();
        return 0;
    };
    if (deltas(h->block_rperm, Er, L.rdrow, &L.rvd, &L.dstride_r)) return -1;
    if (deltas(h->block_cperm, Ec, L.cdrow, &L.cvd, &L.dstride_c)) return -1;
    L.nd_r = (int)(L.dstride_r / NT);
    L.nd_c = (int)(L.dstride_c / NT);
    L.er = Er;
    L.ec = Ec;
    return h->delta_scale ? build_unit_codes(h, rv, cv) : 0;
}

// Shared-matrix MFMA layout (pdhg_mfma.hip).  Planner: the smallest tile grid (16 TM rows x 16 TN
// columns) holding the matrix; used by AUTO when the matrix is the same in every scenario and
// fills at least 1/16 of the padded tiles (below that the dense products waste more than 15 of 16
// MFMA lanes and the sparse layouts win).  Returns 0 (chosen), 1 (does not fit / not chosen).
static constexpr int kMfmaMinScenarios = 4096;

static int pick_mfma_variant(const phg_batch* b, bool shared, bool forced, int* shape) {
    if (!shared) return -1;
    for (int v = 0; v < pdhg_mfma_num_variants(); ++v) {
        int sh[2];
        pdhg_mfma_variant_shape(v, sh);
        if (b->m > 16 * sh[0] || b->n > 16 * sh[1]) continue;
        if (!forced && 16L * b->nnz < 256L * sh[0] * sh[1]) return -1;   // density rule
        // size rule: 16 scenarios per wave means S / 16 waves; below ~one wave per CU the
        // one-scenario-per-wave kernels finish sooner (their PDHG iteration is shorter and they
        // spread over more SIMDs).  Measured on hydro trees (MI355X): S = 2 000 gather 0.240 ms vs
        // MFMA 0.368 ms per launch; S = 20 000 gather 1.018 ms vs MFMA 0.426 ms
        if (!forced && b->S < kMfmaMinScenarios) return -1;
        shape[0] = sh[0];
        shape[1] = sh[1];
        return v;
    }
    return -1;
}

// Fragments of the SCALED shared matrix (scenario 0's values after prep: every scenario's are the
// same, prep being deterministic on identical input) in the order pdhg_mfma_kernel reads them.
static int build_mfma_fragments(phg_handle* h, const phg_batch* b) {
    const int TM = h->mshape[0], TN = h->mshape[1], NF = 4 * TM * TN;
    const int M = 16 * TM, N = 16 * TN;
    std::vector<double> v0(b->nnz);
    CK(hipMemcpyAsync(v0.data(), h->vals, b->nnz * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CK(hipStreamSynchronize(h->stream));
    std::vector<double> A((size_t)M * N, 0.0);
    for (int i = 0; i < b->m; ++i)
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) A[(size_t)i * N + b->colidx[p]] = v0[p];
    std::vector<double> fr((size_t)2 * NF * 64, 0.0);
    unsigned long long nza = 0, nzb = 0;
    for (int t = 0; t < TM; ++t)
        for (int u = 0; u < TN; ++u)
            for (int j = 0; j < 4; ++j) {
                const int fa = (t * TN + u) * 4 + j, fb = (u * TM + t) * 4 + j;
                for (int l = 0; l < 64; ++l) {
                    // A x: A[16 t + (l & 15)][16 u + 4 j + (l >> 4)]
                    const double va = A[(size_t)(16 * t + (l & 15)) * N + 16 * u + 4 * j + (l >> 4)];
                    // A^T y: A[16 t + 4 j + (l >> 4)][16 u + (l & 15)]
                    const double vb = A[(size_t)(16 * t + 4 * j + (l >> 4)) * N + 16 * u + (l & 15)];
                    fr[(size_t)fa * 64 + l] = va;
                    fr[(size_t)(NF + fb) * 64 + l] = vb;
                    if (va != 0.0) nza |= 1ull << fa;
                    if (vb != 0.0) nzb |= 1ull << fb;
                }
            }
    double* d;
    if (dput(h, &d, fr.data(), fr.size())) return -1;
    h->mf.frag = d;
    h->mf.nz_ax = nza;
    h->mf.nz_aty = nzb;
    return 0;
}

// Bordered block-diagonal layout (pdhg_border.hip).  Columns linked by "sparse" rows (at most
// max(16, 4 x the mean row length) nonzeros) form blocks (union-find); the blocks are packed,
// heaviest first, into K groups of about equal nonzeros; rows inside one group are local to it, the
// others are linking rows (at most 1024).  K: the smallest with every group's slice in LDS, raised
// to fill the chip when there are few scenarios (at most 16).  Returns 1 (not applicable) when the
// matrix has no such structure -- fewer than two blocks, a dominant block, too many linking rows or
// no K that fits -- and the range-split streaming kernel is used instead.
static int uf_find(std::vector<int>& p, int x) {
    while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
    return x;
}

static int pad4(int len) { return (len + 3) & ~3; }

static int build_border_layout(phg_handle* h, const phg_batch* b, const std::vector<int>& colptr,
                               const std::vector<int>& csc_row, const std::vector<int>& csc_p, int cap) {
    const int n = b->n, m = b->m, S = std::max(1, b->S);
    const int* rp = b->rowptr;
    const int* ci = b->colidx;
    const int thr = std::max(16, (int)(4.0 * (double)b->nnz / std::max(1, m)));
    std::vector<int> par(n);
    for (int j = 0; j < n; ++j) par[j] = j;
    for (int i = 0; i < m; ++i) {
        if (rp[i + 1] - rp[i] > thr || rp[i + 1] == rp[i]) continue;
        const int r0 = uf_find(par, ci[rp[i]]);
        for (int p = rp[i] + 1; p < rp[i + 1]; ++p) {
            const int r = uf_find(par, ci[p]);
            if (r != r0) par[r] = r0;
        }
    }
    std::vector<int> cid(n, -1), root_id(n, -1);
    std::vector<long> wt;
    for (int j = 0; j < n; ++j) {
        const int r = uf_find(par, j);
        if (root_id[r] < 0) { root_id[r] = (int)wt.size(); wt.push_back(0); }
        cid[j] = root_id[r];
        wt[cid[j]] += colptr[j + 1] - colptr[j] + 1;
    }
    const int ncomp = (int)wt.size();
    if (ncomp < 2) return 1;
    std::vector<int> by(ncomp);
    for (int c = 0; c < ncomp; ++c) by[c] = c;
    std::stable_sort(by.begin(), by.end(), [&](int x, int y) { return wt[x] > wt[y]; });
    long total = 0;
    for (long w : wt) total += w;

    BorderLayout& B = h->bd;
    const size_t budget = 156 * 1024;
    const char* eregs = std::getenv("PHG_BORDER_REG");   // 0: memory-resident variant only
    const bool allow_reg = !(eregs && std::atoi(eregs) == 0);
    std::vector<int> gof(n), rgrp(m), linkidx(m, -1);
    std::vector<BorderGroup> groups;
    std::vector<int> link_rows;
    auto plan = [&](int K, long* gmax) -> size_t {
        std::vector<long> load(K, 0);
        std::vector<int> cg(ncomp);
        for (int c : by) {
            int k = 0;
            for (int q = 1; q < K; ++q)
                if (load[q] < load[k]) k = q;
            cg[c] = k;
            load[k] += wt[c];
        }
        *gmax = *std::max_element(load.begin(), load.end());
        for (int j = 0; j < n; ++j) gof[j] = cg[cid[j]];
        link_rows.clear();
        std::fill(linkidx.begin(), linkidx.end(), -1);
        for (int i = 0; i < m; ++i) {
            int g = rp[i + 1] > rp[i] ? gof[ci[rp[i]]] : 0;
            for (int p = rp[i]; p < rp[i + 1]; ++p)
                if (gof[ci[p]] != g) { g = -1; break; }
            rgrp[i] = g;
            if (g < 0) { linkidx[i] = (int)link_rows.size(); link_rows.push_back(i); }
        }
        B.nlink = (int)link_rows.size();
        if (B.nlink > 1024) return SIZE_MAX;
        // entry counts per group, and padded to 4 per row / column segment (register variant)
        std::vector<int> nc(K, 0), nr(K, 0), nrz(K, 0), nlz(K, 0), ncz(K, 0), nrz4(K, 0), nlz4(K, 0), ncz4(K, 0);
        std::vector<int> lcnt(K, 0);
        for (int j = 0; j < n; ++j) {
            const int len = colptr[j + 1] - colptr[j];
            nc[gof[j]]++;
            ncz[gof[j]] += len;
            ncz4[gof[j]] += pad4(len);
        }
        for (int i = 0; i < m; ++i) {
            if (rgrp[i] >= 0) {
                nr[rgrp[i]]++;
                nrz[rgrp[i]] += rp[i + 1] - rp[i];
                nrz4[rgrp[i]] += pad4(rp[i + 1] - rp[i]);
            } else {
                std::fill(lcnt.begin(), lcnt.end(), 0);
                for (int p = rp[i]; p < rp[i + 1]; ++p) lcnt[gof[ci[p]]]++;
                for (int k = 0; k < K; ++k) { nlz[k] += lcnt[k]; nlz4[k] += pad4(lcnt[k]); }
            }
        }
        auto vmax = [](const std::vector<int>& v) { return *std::max_element(v.begin(), v.end()); };
        B.C_max = vmax(nc);
        B.R_max = vmax(nr);
        // register-resident variant (at most 2 owned columns and 2 rows per thread of 512)
        const int per = std::max(B.C_max, B.R_max);
        B.reg = (allow_reg && per <= pdhg_border_max_per_thread()) ? 2 : 0;
        size_t bytes = SIZE_MAX;
        if (B.reg) {   // padded segments; an even count of doubles ahead of the (16-byte) int region
            B.nrz_max = vmax(nrz4);
            B.nlz_max = vmax(nlz4);
            B.ncz_max = vmax(ncz4);
            B.xtmp_len = std::max(B.nlink + K, 16 * K);
            B.xtmp_len += (B.C_max + B.R_max + B.nlink + B.xtmp_len) & 1;
            bytes = pdhg_border_lds_bytes(B);
            if (bytes > budget) B.reg = 0;   // the memory-resident variant needs less LDS
        }
        if (!B.reg) {
            B.nrz_max = vmax(nrz);
            B.nlz_max = vmax(nlz);
            B.ncz_max = vmax(ncz);
            B.xtmp_len = std::max(B.nlink + K, 16 * K);
            bytes = pdhg_border_lds_bytes(B);
        }
        return bytes;
    };
    long gmax = 0;
    int K = 0;
    if (const char* ek = std::getenv("PHG_STREAM_K")) {
        K = std::max(1, std::min(cap, std::atoi(ek)));
        if (plan(K, &gmax) > budget) return 1;
    } else {
        // smallest K with the register-resident variant (K <= 32), else the smallest K <= 16 that
        // fits the memory-resident one; then more workgroups per scenario while that fills the
        // chip better (few scenarios), keeping the variant
        int K_any = 0;
        for (int k = 1; k <= 32 && K == 0; ++k)
            if (plan(k, &gmax) <= budget) {
                if (!K_any && k <= 16) K_any = k;
                if (B.reg) K = k;
            }
        if (K == 0) K = K_any;
        if (K == 0) return 1;
        const bool reg_at_K = (plan(K, &gmax), B.reg != 0);
        const int fill = std::min(reg_at_K ? 32 : 16, cap / S);
        if (fill > K && plan(fill, &gmax) <= budget && (B.reg != 0) == reg_at_K) K = fill;
        else plan(K, &gmax);
    }
    // a dominant block leaves the other workgroups idle: not this layout's shape
    if (K > 1 && (double)gmax > 2.0 * (double)total / K) return 1;

    // concatenated per-group arrays
    std::vector<int> col_list, row_list, rptr, rcol, rperm, lptr, lcol, lperm, cptr, crow, cperm;
    std::vector<int> rcl, lcl, crl, lpos_col(n, -1), lpos_row(m, -1);
    // the register variant's segments are padded to 4 entries (position -1: value 0, index 0) for its
    // 4-wide gathers (pdhg_border.hip); the memory-resident kernel reads them unpadded
    const bool pad = B.reg != 0;
    groups.assign(K, BorderGroup{});
    for (int k = 0; k < K; ++k) {
        BorderGroup& G = groups[k];
        G.c0 = (int)col_list.size();
        for (int j = 0; j < n; ++j)
            if (gof[j] == k) col_list.push_back(j);
        G.nc = (int)col_list.size() - G.c0;
        for (int q = 0; q < G.nc; ++q) lpos_col[col_list[G.c0 + q]] = q;
        G.r0 = (int)row_list.size();
        for (int i = 0; i < m; ++i)
            if (rgrp[i] == k) row_list.push_back(i);
        G.nr = (int)row_list.size() - G.r0;
        for (int q = 0; q < G.nr; ++q) lpos_row[row_list[G.r0 + q]] = q;
        G.rp0 = (int)rptr.size();
        G.rz0 = (int)rcol.size();
        for (int q = 0; q < G.nr; ++q) {
            const int i = row_list[G.r0 + q];
            rptr.push_back((int)rcol.size() - G.rz0);
            for (int p = rp[i]; p < rp[i + 1]; ++p) { rcol.push_back(ci[p]); rcl.push_back(lpos_col[ci[p]]); rperm.push_back(p); }
            while (pad && ((int)rcol.size() - G.rz0) % 4) { rcol.push_back(0); rcl.push_back(0); rperm.push_back(-1); }
        }
        rptr.push_back((int)rcol.size() - G.rz0);
        G.nrz = (int)rcol.size() - G.rz0;
        G.lp0 = (int)lptr.size();
        G.lz0 = (int)lcol.size();
        for (int l = 0; l < B.nlink; ++l) {
            const int i = link_rows[l];
            lptr.push_back((int)lcol.size() - G.lz0);
            for (int p = rp[i]; p < rp[i + 1]; ++p)
                if (gof[ci[p]] == k) { lcol.push_back(ci[p]); lcl.push_back(lpos_col[ci[p]]); lperm.push_back(p); }
            while (pad && ((int)lcol.size() - G.lz0) % 4) { lcol.push_back(0); lcl.push_back(0); lperm.push_back(-1); }
        }
        lptr.push_back((int)lcol.size() - G.lz0);
        G.nlz = (int)lcol.size() - G.lz0;
        G.cp0 = (int)cptr.size();
        G.cz0 = (int)crow.size();
        for (int q = 0; q < G.nc; ++q) {
            const int j = col_list[G.c0 + q];
            cptr.push_back((int)crow.size() - G.cz0);
            for (int e = colptr[j]; e < colptr[j + 1]; ++e) {
                const int r = csc_row[e];
                crow.push_back(linkidx[r] >= 0 ? -(linkidx[r] + 1) : r);
                crl.push_back(linkidx[r] >= 0 ? -(linkidx[r] + 1) : lpos_row[r]);
                cperm.push_back(csc_p[e]);
            }
            while (pad && ((int)crow.size() - G.cz0) % 4) { crow.push_back(0); crl.push_back(0); cperm.push_back(-1); }
        }
        cptr.push_back((int)crow.size() - G.cz0);
        G.ncz = (int)crow.size() - G.cz0;
    }
    StreamLayout& L = h->st;
    L.K = K;
    L.slots = std::max(1, std::min(S, cap / K));
    L.res = 0;
    BorderGroup* gd;
    if (dput(h, &gd, groups.data(), groups.size())) return -1;
    B.grp = gd;
    int* p;
    auto put_ints = [&](const std::vector<int>& v, const int** dst) {
        if (dput(h, &p, v.data(), v.size())) return -1;
        *dst = p;
        return 0;
    };
    if (put_ints(link_rows, &B.link_rows) || put_ints(col_list, &B.col_list) || put_ints(row_list, &B.row_list) ||
        put_ints(rptr, &B.rptr) || put_ints(rcol, &B.rcol) || put_ints(rperm, &B.rperm) ||
        put_ints(lptr, &B.lptr) || put_ints(lcol, &B.lcol) || put_ints(lperm, &B.lperm) ||
        put_ints(cptr, &B.cptr) || put_ints(crow, &B.crow) || put_ints(cperm, &B.cperm) ||
        put_ints(rcl, &B.rcl) || put_ints(lcl, &B.lcl) || put_ints(crl, &B.crl))
        return -1;
    double* d;
    // (register variant: 8-byte tagged granules, pdhg_border_granule_words)
    if (dalloc(h, &d, std::max((size_t)L.slots * 2 * K * std::max(1, B.nlink), pdhg_border_granule_words(B, L)))) return -1;
    B.plink = d;
    const size_t Sn = (size_t)b->S * n, Sm = (size_t)b->S * m;
    if (dalloc(h, &d, Sn)) return -1; L.cs = d;
    if (dalloc(h, &d, Sn)) return -1; L.qs = d;
    if (dalloc(h, &d, Sn)) return -1; L.lo = d;
    if (dalloc(h, &d, Sn)) return -1; L.hi = d;
    if (dalloc(h, &d, Sn)) return -1; L.xsum = d;
    if (dalloc(h, &d, Sn)) return -1; L.aty = d;
    if (dalloc(h, &d, Sn)) return -1; L.xr = d;
    if (dalloc(h, &d, Sm)) return -1; L.ysum = d;
    if (dalloc(h, &d, Sm)) return -1; L.axo = d;
    if (dalloc(h, &d, Sm)) return -1; L.yr = d;
    if (dalloc(h, &d, (size_t)L.slots * K * 16)) return -1; L.part = d;
    // split solves (pdhg_border.hip): with more scenarios than slots, a solve past slice x
    // check_every iterations during the first pass is suspended and re-queued (PHG_BORDER_SLICE,
    // 0 = off)
    B.slice = 0;
    if (B.reg && b->S > L.slots) {
        B.slice = 8;
        if (const char* es = std::getenv("PHG_BORDER_SLICE")) B.slice = std::max(0, std::atoi(es));
    }
    if (B.slice > 0) {
        int* rq;
        if (dalloc(h, &rq, (size_t)b->S)) return -1;
        B.requeue = rq;
        if (dalloc(h, &d, (size_t)b->S * 8)) return -1;
        B.susp = d;
    }
    unsigned* u;
    if (dalloc(h, &u, (size_t)kCtrlBar + 3 * (size_t)L.slots)) return -1; L.ctrl = u;
    int* e;
    if (dalloc(h, &e, 1)) return -1; L.err = e;
    h->stream_layout = true;
    h->border_layout = true;
    return 0;
}

// Streaming layout (pdhg_stream.hip).  Rows and columns are split into K contiguous ranges of
// about equal nonzeros, one per workgroup of a slot; slots of K co-resident workgroups (one
// 1024-thread workgroup per CU) take scenarios from a queue.  K: the smallest split whose largest
// slice (CSR of the owned rows + CSC of the owned columns) fits in a workgroup's LDS -- the
// resident variant, whose gathers then touch memory only for the published x / y -- raised to
// fill the chip when there are few scenarios (at most 16); when no K <= 16 fits, the streamed
// variant (structure and values read from memory every iteration) with K filling the chip.
static int build_stream_layout(phg_handle* h, const phg_batch* b, const std::vector<int>& colptr,
                               const std::vector<int>& csc_row, const std::vector<int>& csc_p, int pol) {
    int cap = 0;
    CK(pdhg_stream_capacity(&cap));
    const char* eb = std::getenv("PHG_STREAM_BORDER");   // 0: AUTO skips the bordered form
    if (pol == PHG_LAYOUT_BORDER || (pol == PHG_LAYOUT_AUTO && !(eb && std::atoi(eb) == 0))) {
        const int r = build_border_layout(h, b, colptr, csc_row, csc_p, cap);
        if (r <= 0) return r;
        if (pol == PHG_LAYOUT_BORDER)
            return fail("phg_load_batch: no bordered block-diagonal structure that fits (pdhg_border.hip)");
    }
    const int n = b->n, m = b->m, nnz = b->nnz, S = std::max(1, b->S);
    auto split = [&](const int* ptr, int cnt, int K, std::vector<int>& first) {
        first.assign(K + 1, cnt);
        first[0] = 0;
        int q = 1;
        for (int i = 0; i < cnt && q < K; ++i)
            if ((long)ptr[i] * K >= (long)q * ptr[cnt]) first[q++] = i;
        for (; q < K; ++q) first[q] = cnt;
        for (int k = 1; k <= K; ++k) first[k] = std::max(first[k], first[k - 1]);
    };
    StreamLayout& L = h->st;
    std::vector<int> rf, cf;
    auto plan = [&](int K) {   // split for K; fills the per-workgroup maxima, returns the LDS bytes
        split(b->rowptr, m, K, rf);
        split(colptr.data(), n, K, cf);
        L.nr_max = L.nc_max = L.R_max = L.C_max = 0;
        for (int k = 0; k < K; ++k) {
            L.nr_max = std::max(L.nr_max, b->rowptr[rf[k + 1]] - b->rowptr[rf[k]]);
            L.nc_max = std::max(L.nc_max, colptr[cf[k + 1]] - colptr[cf[k]]);
            L.R_max = std::max(L.R_max, rf[k + 1] - rf[k]);
            L.C_max = std::max(L.C_max, cf[k + 1] - cf[k]);
        }
        L.res = 1;
        return pdhg_stream_lds_bytes(L);
    };
    const size_t budget = 156 * 1024;   // 160 KB per CU less the static reduction scratch
    int K = 0, res = 0;
    const char* ek = std::getenv("PHG_STREAM_K");
    const char* er = std::getenv("PHG_STREAM_RES");
    const bool allow_res = !(er && std::atoi(er) == 0);
    if (ek) {
        K = std::max(1, std::min(cap, std::atoi(ek)));
        res = allow_res && plan(K) <= budget;
    } else {
        for (int k = 1; k <= 16 && allow_res && !res; ++k)
            if (plan(k) <= budget) { K = k; res = 1; }
        const int fill = std::max(1, std::min(16, cap / S));
        if (!res) K = fill;
        else if (fill > K) { K = fill; res = plan(K) <= budget; }
    }
    plan(K);
    L.res = res;
    L.K = K;
    L.slots = std::max(1, std::min(S, cap / K));
    if (K > cap) return fail("phg_load_batch: stream layout wants more workgroups per scenario than fit");
    int* p;
    if (dput(h, &p, rf.data(), rf.size())) return -1; L.row_first = p;
    if (dput(h, &p, cf.data(), cf.size())) return -1; L.col_first = p;
    if (dput(h, &p, b->rowptr, m + 1)) return -1; L.rowptr = p;
    if (dput(h, &p, b->colidx, nnz)) return -1; L.colidx = p;
    if (dput(h, &p, colptr.data(), n + 1)) return -1; L.colptr = p;
    if (dput(h, &p, csc_row.data(), nnz)) return -1; L.rowidx = p;
    h->stream_cperm = csc_p;
    const size_t Sn = (size_t)b->S * n, Sm = (size_t)b->S * m;
    double* d;
    if (dalloc(h, &d, Sn)) return -1; L.cs = d;
    if (dalloc(h, &d, Sn)) return -1; L.qs = d;
    if (dalloc(h, &d, Sn)) return -1; L.lo = d;
    if (dalloc(h, &d, Sn)) return -1; L.hi = d;
    if (dalloc(h, &d, Sn)) return -1; L.xsum = d;
    if (dalloc(h, &d, Sn)) return -1; L.aty = d;
    if (dalloc(h, &d, Sn)) return -1; L.xr = d;
    if (dalloc(h, &d, Sm)) return -1; L.ysum = d;
    if (dalloc(h, &d, Sm)) return -1; L.axo = d;
    if (dalloc(h, &d, Sm)) return -1; L.yr = d;
    if (dalloc(h, &d, (size_t)L.slots * K * 16)) return -1; L.part = d;
    unsigned* u;
    if (dalloc(h, &u, (size_t)kCtrlBar + 3 * (size_t)L.slots)) return -1; L.ctrl = u;
    int* e;
    if (dalloc(h, &e, 1)) return -1; L.err = e;
    h->stream_layout = true;
    return 0;
}

// scaled values in CSR order are the handle's own array; the CSC copy is gathered after prep
static int build_stream_values(phg_handle* h) {
    StreamLayout& L = h->st;
    const int Sv = h->vals_shared ? 1 : h->S;
    if (h->border_layout) {   // gathered into LDS through the layout's position arrays
        L.rvals = h->vals;
        L.vstride = h->vals_shared ? 0 : h->nnz;
        return 0;
    }
    int* perm;
    double* cv;
    if (dput(h, &perm, h->stream_cperm.data(), h->stream_cperm.size())) return -1;
    if (dalloc(h, &cv, (size_t)Sv * h->nnz)) return -1;
    CK(piece_gather_launch(h->vals, h->nnz, perm, h->nnz, Sv, cv, h->stream));
    L.rvals = h->vals;
    L.cvals = cv;
    L.vstride = h->vals_shared ? 0 : h->nnz;
    return 0;
}

// ----------------------------------------------------------------------------- value forms
// phg_batch.vals_form: every entry point works on the per-scenario [S*nnz] form; the shared and delta
// forms are expanded here (store holds the expansion, out points into it).  Returns 0 / -1.
static int normalize_vals(const phg_batch* in, phg_batch& out, std::vector<double>& store, const char* who) {
    out = *in;
    if (in->vals_form == PHG_VALS_PER_SCENARIO || !in->vals) return 0;
    if (in->vals_form != PHG_VALS_SHARED && in->vals_form != PHG_VALS_DELTA)
        return fail(std::string(who) + ": unknown vals_form");
    if (in->S <= 0 || in->nnz <= 0) return fail(std::string(who) + ": empty batch");
    const size_t S = (size_t)in->S, nnz = (size_t)in->nnz;
    store.resize(S * nnz);
    for (size_t s = 0; s < S; ++s) std::memcpy(store.data() + s * nnz, in->vals, nnz * sizeof(double));
    if (in->vals_form == PHG_VALS_DELTA) {
        const int nd = in->n_delta;
        if (nd < 0 || (nd > 0 && (!in->delta_pos || !in->delta_vals)))
            return fail(std::string(who) + ": delta form needs n_delta >= 0, delta_pos and delta_vals");
        for (int d = 0; d < nd; ++d) {
            const int p = in->delta_pos[d];
            if (p < 0 || p >= in->nnz || (d > 0 && p <= in->delta_pos[d - 1]))
                return fail(std::string(who) + ": delta_pos must be strictly increasing CSR positions");
        }
        for (size_t s = 0; s < S; ++s)
            for (int d = 0; d < nd; ++d) store[s * nnz + in->delta_pos[d]] = in->delta_vals[s * nd + d];
    }
    out.vals = store.data();
    out.vals_form = PHG_VALS_PER_SCENARIO;
    out.n_delta = 0;
    out.delta_pos = nullptr;
    out.delta_vals = nullptr;
    return 0;
}

// ----------------------------------------------------------------------------- presolve
// Singleton rows (PDLP-style presolve): a row  lo <= a x_j <= hi  with ONE nonzero, on a column
// that is not a nonant, is the column bound  lo/a <= x_j <= hi/a  (swapped for a < 0).  The LP is
// unchanged, but PDHG handles a bound exactly in its projection while a row costs a dual variable
// and its share of every A x / A^T y: on farmer (30 EnforceQuotas rows of 91) the prox-QPs take
// ~38 % fewer PDHG iterations (tools/pdhg_algo_lab.py, LAB_PRESOLVE) and each iteration is cheaper.
// A row is folded only if it is a singleton with a finite nonzero coefficient in EVERY scenario
// (one shared pattern) and the tightened bounds stay consistent; nonant columns keep their rows so
// that fixing nonants (xhat) still sees them.  Row duals of folded rows read back as 0.
struct Presolved {
    phg_batch b{};
    std::vector<int32_t> rowptr, colidx;
    std::vector<double> vals, rl, ru, cl, cu;
    std::vector<int> row_map;
    int removed = 0;
    // the folded rows as column bounds: fold_col[f], and per scenario [fold_lo, fold_hi][f * S + s]
    // (phg_set_col_bounds intersects a caller's new column bounds with them again)
    std::vector<int> fold_col;
    std::vector<double> fold_lo, fold_hi;
};

static void presolve_singletons(const phg_batch* in, Presolved& P) {
    const int S = in->S, n = in->n, m = in->m, nnz = in->nnz;
    P.b = *in;
    P.row_map.resize(m);
    for (int i = 0; i < m; ++i) P.row_map[i] = i;
    P.removed = 0;
    if (!in->vals || !in->row_lo || !in->row_hi || !in->col_lo || !in->col_hi || !in->nonant_col) return;
    std::vector<char> is_nonant(n, 0);
    for (int k = 0; k < in->N; ++k)
        if (in->nonant_col[k] >= 0 && in->nonant_col[k] < n) is_nonant[in->nonant_col[k]] = 1;
    std::vector<int> cand;
    for (int i = 0; i < m; ++i) {
        if (in->rowptr[i + 1] - in->rowptr[i] != 1) continue;
        const int p = in->rowptr[i], j = in->colidx[p];
        if (is_nonant[j]) continue;
        bool ok = true;
        for (int s = 0; s < S && ok; ++s) {
            const double a = in->vals[(size_t)s * nnz + p];
            if (!(a != 0.0) || !std::isfinite(a)) { ok = false; break; }
            double lo = in->row_lo[(size_t)s * m + i] / a, hi = in->row_hi[(size_t)s * m + i] / a;
            if (a < 0) std::swap(lo, hi);
            ok = std::max(in->col_lo[(size_t)s * n + j], lo) <= std::min(in->col_hi[(size_t)s * n + j], hi);
        }
        if (ok) cand.push_back(i);
    }
    if ((int)cand.size() == m) cand.pop_back();   // the kernels want at least one row
    if (cand.empty()) return;
    // two singleton rows on one column both tighten it; check the combined bounds too
    P.cl.assign(in->col_lo, in->col_lo + (size_t)S * n);
    P.cu.assign(in->col_hi, in->col_hi + (size_t)S * n);
    std::vector<char> drop(m, 0);
    for (int i : cand) {
        const int p = in->rowptr[i], j = in->colidx[p];
        bool ok = true;
        for (int s = 0; s < S && ok; ++s) {
            const double a = in->vals[(size_t)s * nnz + p];
            double lo = in->row_lo[(size_t)s * m + i] / a, hi = in->row_hi[(size_t)s * m + i] / a;
            if (a < 0) std::swap(lo, hi);
            ok = std::max(P.cl[(size_t)s * n + j], lo) <= std::min(P.cu[(size_t)s * n + j], hi);
        }
        if (!ok) continue;
        P.fold_col.push_back(j);
        for (int s = 0; s < S; ++s) {
            const double a = in->vals[(size_t)s * nnz + p];
            double lo = in->row_lo[(size_t)s * m + i] / a, hi = in->row_hi[(size_t)s * m + i] / a;
            if (a < 0) std::swap(lo, hi);
            double& L = P.cl[(size_t)s * n + j];
            double& U = P.cu[(size_t)s * n + j];
            L = std::max(L, lo);
            U = std::min(U, hi);
            P.fold_lo.push_back(lo);
            P.fold_hi.push_back(hi);
        }
        drop[i] = 1;
        ++P.removed;
    }
    if (!P.removed) return;
    const int m2 = m - P.removed;
    P.rowptr.assign(1, 0);
    std::vector<int> keep_p;
    for (int i = 0, r = 0; i < m; ++i) {
        if (drop[i]) { P.row_map[i] = -1; continue; }
        P.row_map[i] = r++;
        for (int q = in->rowptr[i]; q < in->rowptr[i + 1]; ++q) {
            P.colidx.push_back(in->colidx[q]);
            keep_p.push_back(q);
        }
        P.rowptr.push_back((int)P.colidx.size());
    }
    const int nnz2 = (int)keep_p.size();
    P.vals.resize((size_t)S * nnz2);
    P.rl.resize((size_t)S * m2);
    P.ru.resize((size_t)S * m2);
    for (int s = 0; s < S; ++s) {
        for (int q = 0; q < nnz2; ++q) P.vals[(size_t)s * nnz2 + q] = in->vals[(size_t)s * nnz + keep_p[q]];
        for (int i = 0; i < m; ++i)
            if (P.row_map[i] >= 0) {
                P.rl[(size_t)s * m2 + P.row_map[i]] = in->row_lo[(size_t)s * m + i];
                P.ru[(size_t)s * m2 + P.row_map[i]] = in->row_hi[(size_t)s * m + i];
            }
    }
    P.b.m = m2;
    P.b.nnz = nnz2;
    P.b.rowptr = P.rowptr.data();
    P.b.colidx = P.colidx.data();
    P.b.vals = P.vals.data();
    P.b.row_lo = P.rl.data();
    P.b.row_hi = P.ru.data();
    P.b.col_lo = P.cl.data();
    P.b.col_hi = P.cu.data();
}

// Column bounds implied by the rows (for phg_opts.safe_bound, bound.hip), per scenario on the caller's
// (presolved, unscaled) data: every INFINITE column bound that a row with a finite side and finite
// activity bounds on its other columns caps is replaced by that cap, widened by a relative 1e-9 of the
// terms involved (round-off of the activity sums: the box must contain every feasible point; a looser
// box only weakens the bound by its reduced cost times the slack).  Passes repeat while a bound turned
// finite (at most 8).  Finite bounds are kept as given.  free_cols: columns left with an infinite side
// in at least one scenario.
static void implied_bounds(const phg_batch* b, std::vector<double>& L, std::vector<double>& U,
                           std::vector<int>& free_cols) {
    const int S = b->S, n = b->n, m = b->m, nnz = b->nnz;
    L.assign(b->col_lo, b->col_lo + (size_t)S * n);
    U.assign(b->col_hi, b->col_hi + (size_t)S * n);
    std::vector<char> free_any(n, 0);
    auto one = [&](int s, std::vector<char>& fr) {
        double* l = L.data() + (size_t)s * n;
        double* u = U.data() + (size_t)s * n;
        const double* v = b->vals + (size_t)s * nnz;
        const double* rlo = b->row_lo + (size_t)s * m;
        const double* rhi = b->row_hi + (size_t)s * m;
        auto fin_ = [](double x) { return std::fabs(x) < 1e300; };
        for (int pass = 0; pass < 8; ++pass) {
            bool changed = false;
            for (int i = 0; i < m; ++i) {
                const double lo = rlo[i], hi = rhi[i];
                if (!fin_(lo) && !fin_(hi)) continue;
                double mn = 0.0, mx = 0.0, mag = 0.0;
                int nmn = 0, nmx = 0;
                for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) {
                    const double a = v[p];
                    const int j = b->colidx[p];
                    if (a == 0.0) continue;
                    const double lmin = a > 0 ? l[j] : u[j], lmax = a > 0 ? u[j] : l[j];
                    if (fin_(lmin)) { mn += a * lmin; mag += std::fabs(a * lmin); } else ++nmn;
                    if (fin_(lmax)) { mx += a * lmax; mag += std::fabs(a * lmax); } else ++nmx;
                }
                if ((nmn > 1 || !fin_(hi)) && (nmx > 1 || !fin_(lo))) continue;
                for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) {
                    const double a = v[p];
                    const int j = b->colidx[p];
                    if (a == 0.0 || (fin_(l[j]) && fin_(u[j]))) continue;
                    const double lmin = a > 0 ? l[j] : u[j], lmax = a > 0 ? u[j] : l[j];
                    // a x_j <= hi - min activity of the other columns
                    if (fin_(hi) && nmn - (fin_(lmin) ? 0 : 1) == 0) {
                        const double rest = mn - (fin_(lmin) ? a * lmin : 0.0);
                        const double cap = (hi - rest) / a;
                        const double sl = 1e-9 * (std::fabs(cap) + (std::fabs(hi) + mag) / std::fabs(a)) + 1e-12;
                        if (a > 0 && !fin_(u[j]) && fin_(cap)) { u[j] = cap + sl; changed = true; }
                        if (a < 0 && !fin_(l[j]) && fin_(cap)) { l[j] = cap - sl; changed = true; }
                    }
                    // a x_j >= lo - max activity of the other columns
                    if (fin_(lo) && nmx - (fin_(lmax) ? 0 : 1) == 0) {
                        const double rest = mx - (fin_(lmax) ? a * lmax : 0.0);
                        const double cap = (lo - rest) / a;
                        const double sl = 1e-9 * (std::fabs(cap) + (std::fabs(lo) + mag) / std::fabs(a)) + 1e-12;
                        if (a > 0 && !fin_(l[j]) && fin_(cap)) { l[j] = cap - sl; changed = true; }
                        if (a < 0 && !fin_(u[j]) && fin_(cap)) { u[j] = cap + sl; changed = true; }
                    }
                }
            }
            if (!changed) break;
        }
        for (int j = 0; j < n; ++j)
            if (!fin_(l[j]) || !fin_(u[j])) fr[j] = 1;
    };
    const int nt = std::max(1, std::min<int>(16, std::min<int>((int)std::thread::hardware_concurrency(), S / 64 + 1)));
    std::vector<std::vector<char>> fr(nt, std::vector<char>(n, 0));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] { for (int s2 = t; s2 < S; s2 += nt) one(s2, fr[t]); });
    for (auto& x : th) x.join();
    for (int t = 0; t < nt; ++t)
        for (int j = 0; j < n; ++j) free_any[j] |= fr[t][j];
    free_cols.clear();
    for (int j = 0; j < n; ++j)
        if (free_any[j]) free_cols.push_back(j);
}

// the presolved batch as the handle keeps it on the host (phg_batch view: pattern, values, bounds)
static phg_batch host_view(const phg_handle* h) {
    phg_batch v{};
    v.S = h->S; v.n = h->n; v.m = h->m; v.nnz = h->nnz; v.N = h->N;
    v.rowptr = h->hb.rowptr.data();
    v.colidx = h->hb.colidx.data();
    v.nonant_col = h->hb.nonant_col.data();
    v.vals = h->hb.vals.data();
    v.row_lo = h->hb.rl.data();
    v.row_hi = h->hb.ru.data();
    v.col_lo = h->hb.cl.data();
    v.col_hi = h->hb.cu.data();
    return v;
}

// the safe-bound pass's implied column bounds and repair candidates, from the current bounds
static int implied_bounds_upload(phg_handle* h) {
    const phg_batch v = host_view(h);
    std::vector<double> il, ih;
    std::vector<int> fc;
    implied_bounds(&v, il, ih, fc);
    SafeBoundArgs& sb = h->sb;
    if (!sb.ilo) {
        double* dp;
        int* ip;
        if (dalloc(h, &dp, il.size())) return -1; sb.ilo = dp;
        if (dalloc(h, &dp, ih.size())) return -1; sb.ihi = dp;
        if (dalloc(h, &ip, std::max(1, h->n))) return -1; sb.free_col = ip;
    }
    CK(hipMemcpyAsync(const_cast<double*>(sb.ilo), il.data(), il.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
    CK(hipMemcpyAsync(const_cast<double*>(sb.ihi), ih.data(), ih.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
    sb.nf = (int)fc.size();
    if (!fc.empty())
        CK(hipMemcpyAsync(const_cast<int*>(sb.free_col), fc.data(), fc.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
    CK(hipStreamSynchronize(h->stream));   // (the host vectors go out of scope)
    h->sb_stale = false;
    return 0;
}

int phg_implied_bounds(const phg_batch* b_in, double* lo, double* hi, int32_t* n_free) {
    if (!b_in || !lo || !hi) return fail("phg_implied_bounds: null argument");
    phg_batch bx;
    std::vector<double> vstore;
    if (normalize_vals(b_in, bx, vstore, "phg_implied_bounds")) return -1;
    const phg_batch* b = &bx;
    if (b->S <= 0 || b->n <= 0 || b->m <= 0 || !b->rowptr || !b->colidx || !b->vals || !b->col_lo ||
        !b->col_hi || !b->row_lo || !b->row_hi)
        return fail("phg_implied_bounds: incomplete batch");
    std::vector<double> L, U;
    std::vector<int> fc;
    implied_bounds(b, L, U, fc);
    std::memcpy(lo, L.data(), L.size() * sizeof(double));
    std::memcpy(hi, U.data(), U.size() * sizeof(double));
    if (n_free) *n_free = (int32_t)fc.size();
    return 0;
}

int phg_set_presolve(phg_handle* h, int32_t on) {
    if (!h) return fail("phg_set_presolve: null handle");
    if (h->loaded) return fail("phg_set_presolve: call before phg_load_batch");
    h->presolve = on ? 1 : 0;
    return 0;
}

int phg_presolve_info(phg_handle* h, int32_t* out2) {
    if (!h || !h->loaded || !out2) return fail("phg_presolve_info: no batch loaded");
    out2[0] = h->m_orig - h->m;
    out2[1] = h->m;
    return 0;
}

int phg_plan(const phg_batch* b_in, int32_t* out8) {
    if (!b_in || !out8) return fail("phg_plan: null argument");
    if (b_in->n <= 0 || b_in->m <= 0 || !b_in->rowptr || !b_in->colidx) return fail("phg_plan: empty pattern");
    phg_batch bx;
    std::vector<double> vstore;
    if (normalize_vals(b_in, bx, vstore, "phg_plan")) return -1;
    Presolved P;   // the plan of what phg_load_batch would run (default policy: presolve on)
    presolve_singletons(&bx, P);
    const phg_batch* b = &P.b;
    LocalPlan plan;
    int sh[4] = {0, 0, 0, 0};
    const int v = pick_local_variant(b, plan, sh);
    if (v == -2) return -1;
    for (int i = 0; i < 8; ++i) out8[i] = 0;
    out8[0] = v;
    if (v >= 0) {
        int ncpl = 0;
        for (int i : plan.cpl_row) ncpl += i >= 0;
        out8[1] = sh[0]; out8[2] = sh[1]; out8[3] = sh[2]; out8[4] = sh[3]; out8[5] = ncpl;
        int lanes = 0;
        for (int l = 0; l < sh[0]; ++l) {
            bool used = false;
            for (int k = 0; k < sh[1]; ++k) used |= plan.col_of[l * sh[1] + k] >= 0;
            lanes += used;
        }
        out8[6] = lanes;
        unsigned mb, mc;
        local_slot_masks(plan, sh, &mb, &mc);
        const unsigned long long bi = local_inf_mask(b, plan, sh[0], sh[1], sh[2], sh[3]);
        const unsigned long long bf = local_fin_mask(b, plan, sh[0], sh[1], sh[2], sh[3]);
        const unsigned qm = local_quad_mask(b, plan, sh[0], sh[1]);
        out8[7] = pdhg_local_pick_masked(v, mb, mc, bi, bf, qm);
        if (const char* e = std::getenv("PHG_LOCAL_DEBUG"); e && std::atoi(e))
            fprintf(stderr, "phg_plan: shape %d x %d x %d x %d MB 0x%x MC 0x%x BI 0x%llx BF 0x%llx QM 0x%x variant %d\n",
                    sh[0], sh[1], sh[2], sh[3], mb, mc, bi, bf, qm, out8[7]);
    }
    return 0;
}

int phg_load_batch(phg_handle* h, const phg_batch* b_arg) {
    if (!h || !b_arg) return fail("phg_load_batch: null argument");
    if (!b_arg->vals) return fail("phg_load_batch: no values");
    phg_batch bx;
    std::vector<double> vstore;
    if (normalize_vals(b_arg, bx, vstore, "phg_load_batch")) return -1;
    const phg_batch* b_in = &bx;
    const phg_batch* b = b_in;
    if (h->loaded) return fail("phg_load_batch: handle already holds a batch");
    if (b->S <= 0 || b->n <= 0 || b->m <= 0 || b->nnz <= 0 || b->N <= 0 || b->L <= 0)
        return fail("phg_load_batch: empty batch");
    if (b->rowptr[0] != 0 || b->rowptr[b->m] != b->nnz) return fail("phg_load_batch: bad rowptr");
    for (int i = 0; i < b->m; ++i) {
        if (b->rowptr[i + 1] < b->rowptr[i]) return fail("phg_load_batch: rowptr not monotone");
        for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) {
            if (b->colidx[p] < 0 || b->colidx[p] >= b->n) return fail("phg_load_batch: colidx out of range");
            if (p > b->rowptr[i] && b->colidx[p] <= b->colidx[p - 1])
                return fail("phg_load_batch: colidx must be strictly increasing inside a row");
        }
    }
    for (int k = 0; k < b->N; ++k)
        if (b->nonant_col[k] < 0 || b->nonant_col[k] >= b->n) return fail("phg_load_batch: nonant_col out of range");
    Presolved P;
    if (h->presolve) presolve_singletons(b_in, P);
    else { P.row_map.resize(b_in->m); for (int i = 0; i < b_in->m; ++i) P.row_map[i] = i; P.b = *b_in; }
    b = &P.b;
    h->m_orig = b_in->m;
    h->row_map = P.row_map;
    CK(hipSetDevice(h->device));
    const int S = b->S, n = b->n, m = b->m, nnz = b->nnz, N = b->N;
    h->S = S; h->n = n; h->m = m; h->nnz = nnz; h->N = N; h->L = b->L; h->N_tot = b->N_tot;
    // the folded PH update by default (no PHG_FOLD / phg_set_fold before the load): it pays where
    // the update streams (S N = 1e8: 477 vs 650 us per update) and, with the round-4 prologue, on the
    // latency-bound farmer 10k too (0.3108 vs 0.3138 ms per PH iteration)
    if (h->fold < 0) h->fold = 1;
    h->n_nodes = b->n_nodes; h->P = std::max(1, b->virt_nproc);
    h->n_pad = (n + 1) & ~1;
    h->sense = b->sense >= 0 ? 1.0 : -1.0;
    // CSC of the shared pattern
    std::vector<int> colptr(n + 1, 0), csc_row(nnz), csc_p(nnz), row_of_p(nnz);
    for (int p = 0; p < nnz; ++p) colptr[b->colidx[p] + 1]++;
    for (int j = 0; j < n; ++j) colptr[j + 1] += colptr[j];
    {
        std::vector<int> fill(colptr.begin(), colptr.end() - 1);
        for (int i = 0; i < m; ++i)
            for (int p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p) {
                const int e = fill[b->colidx[p]]++;
                csc_row[e] = i;
                csc_p[e] = p;
                row_of_p[p] = i;
            }
    }
    {
        std::vector<int> col_nonant(n, -1);
        for (int k = 0; k < b->N; ++k) col_nonant[b->nonant_col[k]] = k;
        int* p;
        if (dput(h, &p, col_nonant.data(), col_nonant.size())) return -1;
        h->lay.col_nonant = p;
    }
    // one matrix for all scenarios? (then the block kernel streams a single copy, and the MFMA
    // layout applies)
    {   // ... and which positions vary (the delta form, whatever form the caller passed)
        const size_t nz = (size_t)b->nnz;
        h->vary.assign(nz, 0);
        for (int s2 = 1; s2 < b->S; ++s2) {
            const double* v = b->vals + s2 * nz;
            for (size_t p = 0; p < nz; ++p) h->vary[p] |= (char)(v[p] != b->vals[p]);
        }
        h->n_vary = 0;
        for (size_t p = 0; p < nz; ++p) h->n_vary += h->vary[p];
        h->vals_shared = h->n_vary == 0;
    }
    // layout: shared-matrix MFMA > lane-local (block-structured patterns) > wave gather
    // (n, m <= 256) > workgroup block
    int lr = 1, gr = 1, br = 1;
    const int pol = h->layout_policy;
    if (pol == PHG_LAYOUT_AUTO || pol == PHG_LAYOUT_MFMA) {
        h->mfma_variant = pick_mfma_variant(b, h->vals_shared, pol == PHG_LAYOUT_MFMA, h->mshape);
        if (h->mfma_variant < 0 && pol == PHG_LAYOUT_MFMA)
            return fail(h->vals_shared ? "phg_load_batch: the matrix does not fit the MFMA tile (n, m <= 16)"
                                       : "phg_load_batch: the MFMA layout needs one matrix shared by all scenarios");
        if (h->mfma_variant >= 0) lr = gr = br = 0;
    }
    if (h->mfma_variant < 0 && (pol == PHG_LAYOUT_AUTO || pol == PHG_LAYOUT_LOCAL)) {
        lr = build_local_layout(h, b, pol == PHG_LAYOUT_LOCAL);
        if (lr < 0) return -1;
        if (lr > 0 && pol == PHG_LAYOUT_LOCAL) return -1;
    }
    if (h->mfma_variant < 0 && lr != 0 && (pol == PHG_LAYOUT_AUTO || pol == PHG_LAYOUT_GATHER)) {
        gr = build_layout(h, b, colptr, csc_row, csc_p);
        if (gr < 0 || (gr > 0 && pol == PHG_LAYOUT_GATHER)) return -1;
    }
    // the one-wave-per-scenario layout only on request: measured on sslp 4 096 it is 1.6x slower than
    // the workgroup kernel (8.86 vs 14.2 ms per PH iteration, the same PDHG iterations)
    int wr = 1;
    if (h->mfma_variant < 0 && lr != 0 && gr != 0 && pol == PHG_LAYOUT_WAVE) {
        wr = build_wave_layout(h, b, colptr, csc_row, csc_p);
        if (wr < 0) return -1;
        if (wr > 0 && pol == PHG_LAYOUT_WAVE)
            return fail("phg_load_batch: the wave layout needs one matrix shared by all scenarios, <= 2 entries "
                        "per column and n <= 1024, m <= 64");
        if (wr == 0) h->variant = -1;
    }
    if (h->mfma_variant < 0 && lr != 0 && gr != 0 && wr != 0 && pol != PHG_LAYOUT_STREAM && pol != PHG_LAYOUT_BORDER) {
        // few varying entries: the constant ones as ONE unscaled copy, each scenario's scaling applied
        // on the fly, only the varying ones streamed per scenario (build_block_values, BlockLayout::vscale)
        const char* ed = std::getenv("PHG_DELTA");
        const bool delta_off = ed && std::atoi(ed) == 0;
        const bool want_delta = !delta_off && h->n_vary > 0 && 2L * h->n_vary <= (long)b->nnz;
        br = build_block_layout(h, b, colptr, csc_row, csc_p, want_delta);
        if (br > 0 && want_delta) br = build_block_layout(h, b, colptr, csc_row, csc_p, false);
        if (br < 0 || (br > 0 && pol == PHG_LAYOUT_BLOCK)) return -1;
        h->variant = -1;
        h->delta_scale = br == 0 && h->bshape[8] != 0;
    }
    if (h->mfma_variant < 0 && lr != 0 && gr != 0 && wr != 0 && br != 0) {
        if (build_stream_layout(h, b, colptr, csc_row, csc_p, pol)) return -1;
        h->variant = -1;
    }
    if (h->mfma_variant >= 0) h->variant = -1;
    // min-form objective
    std::vector<double> cmin((size_t)S * n), off((size_t)S, 0.0);
    for (size_t e = 0; e < cmin.size(); ++e) cmin[e] = h->sense * b->c[e];
    if (b->obj_offset)
        for (int s = 0; s < S; ++s) off[s] = h->sense * b->obj_offset[s];
    if (dput(h, &h->vals, b->vals, (size_t)S * nnz)) return -1;
    if (dput(h, &h->c, cmin.data(), cmin.size())) return -1;
    if (dput(h, &h->cl, b->col_lo, (size_t)S * n)) return -1;
    if (dput(h, &h->cu, b->col_hi, (size_t)S * n)) return -1;
    if (dput(h, &h->rl, b->row_lo, (size_t)S * m)) return -1;
    if (dput(h, &h->ru, b->row_hi, (size_t)S * m)) return -1;
    if (dput(h, &h->obj_off, off.data(), S)) return -1;
    if (dalloc(h, &h->dc, (size_t)S * n)) return -1;
    if (dalloc(h, &h->dr, (size_t)S * m)) return -1;
    if (dalloc(h, &h->eta, S)) return -1;
    if (dalloc(h, &h->bnorm, S)) return -1;
    if (dalloc(h, &h->W, (size_t)S * N)) return -1;
    if (dalloc(h, &h->rho, (size_t)S * N)) return -1;
    if (dalloc(h, &h->fixed, (size_t)S * N)) return -1;
    if (dalloc(h, &h->Z, (size_t)S * N)) return -1;
    if (dalloc(h, &h->Psm, (size_t)S * N)) return -1;
    if (dalloc(h, &h->beta, (size_t)S * N)) return -1;
    // xbar and xsqbar adjacent: [xbar | xsqbar] has the node-sum buffer's layout, so the W update of a
    // pending folded update (flush_fold) reads them as its node sums
    if (dalloc(h, &h->xbar, 2 * (size_t)std::max(1, b->N_tot))) return -1;
    h->xsqbar = h->xbar + std::max(1, b->N_tot);
    if (dalloc(h, &h->xs, (size_t)S * n)) return -1;
    if (dalloc(h, &h->ys, (size_t)S * m)) return -1;
    if (dalloc(h, &h->omega, S)) return -1;
    if (dalloc(h, &h->back.xs, (size_t)S * n)) return -1;
    if (dalloc(h, &h->back.ys, (size_t)S * m)) return -1;
    if (dalloc(h, &h->back.omega, S)) return -1;
    if (dalloc(h, &h->back.xN, (size_t)S * N)) return -1;
    if (dalloc(h, &h->back.obj, S)) return -1;
    if (dalloc(h, &h->back.bound, S)) return -1;
    if (dalloc(h, &h->back.kkt, S)) return -1;
    if (dalloc(h, &h->back.iters, S)) return -1;
    if (dalloc(h, &h->back.status, S)) return -1;
    if (dalloc(h, &h->x_out, (size_t)S * n)) return -1;
    if (dalloc(h, &h->y_out, (size_t)S * m)) return -1;
    if (dalloc(h, &h->xN, (size_t)S * N)) return -1;
    if (dalloc(h, &h->obj, S)) return -1;
    if (dalloc(h, &h->bound, S)) return -1;
    if (dalloc(h, &h->kkt, S)) return -1;
    if (dalloc(h, &h->eval, S)) return -1;
    if (dalloc(h, &h->iters, S)) return -1;
    if (dalloc(h, &h->status, S)) return -1;
    if (dalloc(h, &h->iters_acc, S)) return -1;
    if (dalloc(h, &h->order, S)) return -1;
    if (dalloc(h, &h->queue, 2)) return -1;
    h->nonant_col_h.assign(b->nonant_col, b->nonant_col + N);
    {   // rows made constant by fixing the nonants (row_bounds in phg_internal.h)
        std::vector<char> isn(n, 0);
        for (int k = 0; k < N; ++k) isn[b->nonant_col[k]] = 1;
        std::vector<unsigned char> rf(m, 0);
        for (int i = 0; i < m; ++i) {
            bool all = b->rowptr[i + 1] > b->rowptr[i];
            for (int p = b->rowptr[i]; p < b->rowptr[i + 1] && all; ++p) all = isn[b->colidx[p]] != 0;
            rf[i] = all ? 1 : 0;
        }
        if (dput(h, &h->row_fixed, rf.data(), rf.size())) return -1;
    }
    if (dput(h, &h->nonant_col_d, b->nonant_col, N)) return -1;
    if (build_ph_tables(h, b)) return -1;
    h->ph.status = h->status;
    h->ph.Z = h->Z;
    h->ph.beta = h->beta;
    h->ph.xN = h->xN; h->ph.W = h->W; h->ph.rho = h->rho; h->ph.xbar = h->xbar; h->ph.xsqbar = h->xsqbar;
    // preconditioning
    PrepArgs pa{};
    pa.S = S; pa.n = n; pa.m = m; pa.nnz = nnz; pa.ruiz_iters = 10; pa.power_iters = 64;
    int* ip;
    if (dput(h, &ip, b->rowptr, m + 1)) return -1; pa.rowptr = ip;
    if (dput(h, &ip, b->colidx, nnz)) return -1; pa.colidx = ip;
    if (dput(h, &ip, colptr.data(), n + 1)) return -1; pa.colptr = ip;
    if (dput(h, &ip, csc_p.data(), nnz)) return -1; pa.csc_p = ip;
    if (dput(h, &ip, row_of_p.data(), nnz)) return -1; pa.row_of_p = ip;
    double* scratch;
    if (dalloc(h, &scratch, (size_t)S * (2 * n + 2 * m))) return -1;
    // delta form: the pieces take the caller's (unscaled) values; prep scales h->vals in place
    double* raw = nullptr;
    if (h->delta_scale) {
        CK(hipMalloc((void**)&raw, (size_t)S * nnz * sizeof(double)));
        CK(hipMemcpyAsync(raw, h->vals, (size_t)S * nnz * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    }
    pa.vals = h->vals; pa.dc = h->dc; pa.dr = h->dr; pa.cl = h->cl; pa.cu = h->cu; pa.rl = h->rl;
    pa.ru = h->ru; pa.eta = h->eta; pa.bnorm = h->bnorm; pa.scratch = scratch;
    CK(prep_launch(pa, h->stream));
    {   // safe bounds (bound.hip): pattern in CSR / CSC now; the implied column bounds and repair
        // candidates at the first safe-bound solve (implied_bounds_upload: a host pass over the
        // batch that the plugin's one-scenario loads and PH runs without bound reads never need)
        SafeBoundArgs& sb = h->sb;
        sb.rowptr = pa.rowptr; sb.colidx = pa.colidx; sb.colptr = pa.colptr; sb.csc_p = pa.csc_p;
        if (dput(h, &ip, csc_row.data(), nnz)) return -1; sb.rowidx = ip;
        sb.ilo = sb.ihi = nullptr;
        sb.free_col = nullptr;
        sb.nf = 0;
        h->sb_stale = true;
        auto& hb = h->hb;
        hb.rowptr.assign(b->rowptr, b->rowptr + m + 1);
        hb.colidx.assign(b->colidx, b->colidx + nnz);
        hb.nonant_col.assign(b->nonant_col, b->nonant_col + N);
        hb.vals.assign(b->vals, b->vals + (size_t)S * nnz);
        hb.rl.assign(b->row_lo, b->row_lo + (size_t)S * m);
        hb.ru.assign(b->row_hi, b->row_hi + (size_t)S * m);
        hb.cl.assign(b->col_lo, b->col_lo + (size_t)S * n);
        hb.cu.assign(b->col_hi, b->col_hi + (size_t)S * n);
        h->fold_col = P.fold_col;
        h->fold_lo = P.fold_lo;
        h->fold_hi = P.fold_hi;
    }
    if (h->local_variant >= 0) {   // the lane image of the scaled batch (LocalLayout::img)
        const int ni = pdhg_local_image_items(h->local_variant);
        const int D = std::max(1, h->lshape[3]);
        double *img, *cimg;
        if (dalloc(h, &img, (size_t)S * ni * h->lshape[0])) return -1;
        if (dalloc(h, &cimg, (size_t)S * D * 3)) return -1;
        PdhgArgs ia{};
        ia.S = S; ia.n = n; ia.m = m; ia.nnz = nnz;
        ia.loc = h->loc;
        ia.dc = h->dc; ia.c = h->c; ia.cl = h->cl; ia.cu = h->cu; ia.dr = h->dr; ia.rl = h->rl; ia.ru = h->ru;
        ia.vals = h->vals;
        CK(pdhg_local_image_launch(h->local_variant, ia, img, cimg, h->stream));
        h->loc.img = img; h->loc.cimg = cimg; h->loc.ni = ni;
    }
    if (h->block_variant >= 0 && build_block_values(h, raw)) return -1;
    if (raw) {
        CK(hipStreamSynchronize(h->stream));
        CK(hipFree(raw));
    }
    if (h->wave_variant >= 0 && build_wave_values(h)) return -1;
    if (h->mfma_variant >= 0 && build_mfma_fragments(h, b)) return -1;
    if (h->stream_layout && build_stream_values(h)) return -1;
    CK(hipStreamSynchronize(h->stream));
    h->loaded = true;
    return 0;
}

int phg_values_info(phg_handle* h, int32_t* o) {
    if (!h || !h->loaded || !o) return fail("phg_values_info: no batch loaded");
    o[0] = h->n_vary;
    o[1] = h->delta_scale ? (h->bshape[10] ? 2 : 1) : 0;
    o[2] = o[3] = 0;
    if (h->block_variant >= 0) {
        const long E = (long)h->block_rperm.size() + (long)h->block_cperm.size();
        if (h->delta_scale) { o[2] = (int32_t)(h->blk.dstride_r + h->blk.dstride_c); o[3] = (int32_t)E; }
        else if (h->vals_shared) o[3] = (int32_t)E;
        else o[2] = (int32_t)E;
    }
    return 0;
}

int phg_mfma_info(phg_handle* h, int32_t* o) {
    if (!h || !h->loaded || !o) return fail("phg_mfma_info: no batch loaded");
    if (h->mfma_variant < 0) return fail("phg_mfma_info: the batch does not use the MFMA layout");
    o[0] = h->mshape[0];
    o[1] = h->mshape[1];
    o[2] = __builtin_popcountll(h->mf.nz_ax);
    o[3] = __builtin_popcountll(h->mf.nz_aty);
    return 0;
}

int phg_local_info(phg_handle* h, int32_t* o) {
    if (!h || !h->loaded || !o) return fail("phg_local_info: no batch loaded");
    if (h->local_variant < 0) return fail("phg_local_info: the batch does not use the lane-local layout");
    CK(hipSetDevice(h->device));
    // (the variant PH's solves run: the nonants are not fixed there)
    o[0] = h->local_variant_free;
    o[1] = h->lshape[0];
    o[2] = pdhg_local_lone(h->local_variant_free, h->S) ? 1 : 0;
    o[3] = pdhg_local_loop_ops(h->local_variant_free);
    return 0;
}

int phg_info(phg_handle* h, int32_t* o) {
    if (!h || !h->loaded) return fail("phg_info: no batch loaded");
    o[0] = h->S; o[1] = h->n; o[2] = h->m_orig; o[3] = h->nnz; o[4] = h->N; o[5] = h->N_tot;
    if (h->stream_layout) { o[6] = (h->border_layout ? (h->bd.reg ? 600 : 500) : 400) + h->st.K; o[7] = (h->bd.reg ? 512 : 1024) * h->st.K; }
    else if (h->mfma_variant >= 0) { o[6] = 300 + h->mfma_variant; o[7] = 4; }
    else if (h->local_variant >= 0) { o[6] = 100 + h->local_variant; o[7] = h->lshape[0]; }
    else if (h->block_variant >= 0) { o[6] = 200 + h->block_variant; o[7] = h->bshape[0]; }
    else if (h->wave_variant >= 0) { o[6] = 700 + h->wave_variant; o[7] = 64; }
    else { o[6] = h->variant; o[7] = 64; }
    return 0;
}

static double* field_ptr(phg_handle* h, int f, size_t* count) {
    const size_t S = h->S, n = h->n, m = h->m, N = h->N;
    switch (f) {
        case PHG_F_X: *count = S * n; return h->x_out;
        case PHG_F_Y: *count = S * m; return h->y_out;
        case PHG_F_XN: *count = S * N; return h->xN;
        case PHG_F_W: *count = S * N; return h->W;
        case PHG_F_RHO: *count = S * N; return h->rho;
        case PHG_F_XBAR: *count = h->N_tot; return h->xbar;
        case PHG_F_XSQBAR: *count = h->N_tot; return h->xsqbar;
        case PHG_F_OBJ: *count = S; return h->obj;
        case PHG_F_BOUND: *count = S; return h->bound;
        case PHG_F_EVAL: *count = S; return h->eval;
        case PHG_F_KKT: *count = S; return h->kkt;
        case PHG_F_FIXED: *count = S * N; return h->fixed;
        case PHG_F_CONV_PART: *count = 2 * (size_t)h->P + 2; return h->convpart;
        case PHG_F_OMEGA: *count = S; return h->omega;
        case PHG_F_Z: *count = S * N; return h->Z;
        case PHG_F_SMOOTH_P: *count = S * N; return h->Psm;
        case PHG_F_SMOOTH_BETA: *count = S * N; return h->beta;
        default: return nullptr;
    }
}

// a page-locked copy of `bytes` of host data, valid until the copies enqueued from it have run
// (stage_done records that point): pageable uploads are staged and synchronised by the runtime, ~25 us
// each; from pinned memory they are plain stream-ordered DMA
// uploads above this size are not staged (no page-locked copy held per slot): they take the
// synchronous pageable path, whose fixed cost is small beside the copy itself
static constexpr size_t kStageMax = (size_t)16 << 20;

static int stage_upload(phg_handle* h, const void* in, size_t bytes, const void** out) {
    if (bytes > kStageMax) {
        *out = in;
        return 0;
    }
    auto& st = h->up[h->up_next];
    if (st.ev) CK(hipEventSynchronize(st.ev));          // the slot's previous copies have run
    else CK(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
    if (st.cap < bytes) {
        if (st.p) CK(hipHostFree(st.p));
        st.p = nullptr;
        st.cap = 0;
        const size_t cap = std::max(bytes, (size_t)4096);
        CK(hipHostMalloc(&st.p, cap, hipHostMallocDefault));
        st.cap = cap;
    }
    std::memcpy(st.p, in, bytes);
    *out = st.p;
    return 0;
}

static int stage_done(phg_handle* h, size_t bytes) {
    if (bytes > kStageMax) {   // the copies read the caller's memory: done before returning
        CK(hipStreamSynchronize(h->stream));
        return 0;
    }
    CK(hipEventRecord(h->up[h->up_next].ev, h->stream));
    h->up_next = (h->up_next + 1) % 4;
    return 0;
}

int phg_set(phg_handle* h, int32_t f, const double* in) {
    if (!h || !h->loaded) return fail("phg_set: no batch loaded");
    h->tp.mode = 0;   // a fused tail's results are for the state as the solve left it
    if ((f == PHG_F_W || f == PHG_F_XBAR || f == PHG_F_CONV_PART) && flush_fold(h)) return -1;
    size_t cnt = 0;
    double* p = field_ptr(h, f, &cnt);
    if (!p) return fail("phg_set: unknown field");
    if ((f == PHG_F_X || f == PHG_F_Y) && materialize_outputs(h)) return -1;
    CK(hipSetDevice(h->device));
    std::vector<double> packed;
    if (f == PHG_F_Y && h->m != h->m_orig) {   // caller's rows -> kept rows
        packed.resize(cnt);
        for (int s2 = 0; s2 < h->S; ++s2)
            for (int i = 0; i < h->m_orig; ++i)
                if (h->row_map[i] >= 0)
                    packed[(size_t)s2 * h->m + h->row_map[i]] = in[(size_t)s2 * h->m_orig + i];
        in = packed.data();
    }
    const void* staged = nullptr;
    if (stage_upload(h, in, cnt * sizeof(double), &staged)) return -1;
    if (f == PHG_F_XBAR)   // also keep the node-sum buffer consistent
        CK(hipMemcpyAsync(h->nodesum, staged, cnt * sizeof(double), hipMemcpyHostToDevice, h->stream));
    CK(hipMemcpyAsync(p, staged, cnt * sizeof(double), hipMemcpyHostToDevice, h->stream));
    if (f == PHG_F_XN) h->xn_external = true;
    if (f == PHG_F_RHO) {   // rho the same in every scenario? then the W update reads its [N] copy
        bool shared = true;
        for (size_t e = (size_t)h->N; e < cnt && shared; ++e) shared = in[e] == in[e % (size_t)h->N];
        if (shared && !h->rho_k) {
            double* q;
            if (dalloc(h, &q, (size_t)std::max(1, h->N))) return -1;
            h->rho_k = q;
        }
        if (shared) CK(hipMemcpyAsync(h->rho_k, staged, (size_t)h->N * sizeof(double), hipMemcpyHostToDevice, h->stream));
        h->ph.rho_k = shared ? h->rho_k : nullptr;
    }
    return stage_done(h, cnt * sizeof(double));
}

int phg_get(phg_handle* h, int32_t f, double* out) {
    if (!h || !h->loaded) return fail("phg_get: no batch loaded");
    if ((f == PHG_F_W || f == PHG_F_XBAR || f == PHG_F_CONV_PART) && flush_fold(h)) return -1;
    size_t cnt = 0;
    double* p = field_ptr(h, f, &cnt);
    if (!p) return fail("phg_get: unknown field");
    if ((f == PHG_F_X || f == PHG_F_Y) && materialize_outputs(h)) return -1;
    if (f == PHG_F_Y && h->m != h->m_orig) {   // kept rows -> caller's rows (folded rows: 0)
        std::vector<double> packed(cnt);
        CK(hipMemcpyAsync(packed.data(), p, cnt * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        CK(hipStreamSynchronize(h->stream));
        for (int s2 = 0; s2 < h->S; ++s2)
            for (int i = 0; i < h->m_orig; ++i)
                out[(size_t)s2 * h->m_orig + i] =
                    h->row_map[i] >= 0 ? packed[(size_t)s2 * h->m + h->row_map[i]] : 0.0;
        return 0;
    }
    CK(hipMemcpyAsync(out, p, cnt * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CK(hipStreamSynchronize(h->stream));
    return 0;
}

int phg_get_i32(phg_handle* h, int32_t f, int32_t* out) {
    if (!h || !h->loaded) return fail("phg_get_i32: no batch loaded");
    CK(hipSetDevice(h->device));
    if (f == PHG_I_ORDER && sched_flush(h)) return -1;
    int* p = f == PHG_I_ITERS ? h->iters : f == PHG_I_STATUS ? h->status : f == PHG_I_ORDER ? h->order : nullptr;
    if (!p) return fail("phg_get_i32: unknown field");
    CK(hipMemcpyAsync(out, p, (size_t)h->S * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    CK(hipStreamSynchronize(h->stream));
    return 0;
}

int phg_solve_results(phg_handle* h, int32_t* status, int32_t* iters, double* kkt, double* obj,
                      double* bound, double* x) {
    if (!h || !h->loaded) return fail("phg_solve_results: no batch loaded");
    CK(hipSetDevice(h->device));
    if (x && materialize_outputs(h)) return -1;
    const size_t S = (size_t)h->S, nx = (size_t)h->S * h->n;
    const size_t bytes = 2 * S * sizeof(int) + 3 * S * sizeof(double) + (x ? nx * sizeof(double) : 0) + 64;
    if (bytes > kStageMax) {   // large batches: straight into the caller's arrays (no page-locked copy kept)
        if (kkt) CK(hipMemcpyAsync(kkt, h->kkt, S * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        if (obj) CK(hipMemcpyAsync(obj, h->obj, S * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        if (bound) CK(hipMemcpyAsync(bound, h->bound, S * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        if (x) CK(hipMemcpyAsync(x, h->x_out, nx * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        if (status) CK(hipMemcpyAsync(status, h->status, S * sizeof(int), hipMemcpyDeviceToHost, h->stream));
        if (iters) CK(hipMemcpyAsync(iters, h->iters, S * sizeof(int), hipMemcpyDeviceToHost, h->stream));
        CK(hipStreamSynchronize(h->stream));
        return 0;
    }
    auto& st = h->down;
    if (st.cap < bytes) {
        if (st.p) CK(hipHostFree(st.p));
        st.p = nullptr;
        st.cap = 0;
        CK(hipHostMalloc(&st.p, bytes, hipHostMallocDefault));
        st.cap = bytes;
    }
    // doubles first (8-byte aligned), then the two int arrays
    double* d = (double*)st.p;
    int* iv = (int*)(d + 3 * S + (x ? nx : 0));
    CK(hipMemcpyAsync(d, h->kkt, S * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CK(hipMemcpyAsync(d + S, h->obj, S * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CK(hipMemcpyAsync(d + 2 * S, h->bound, S * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (x) CK(hipMemcpyAsync(d + 3 * S, h->x_out, nx * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CK(hipMemcpyAsync(iv, h->status, S * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    CK(hipMemcpyAsync(iv + S, h->iters, S * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    CK(hipStreamSynchronize(h->stream));
    if (kkt) std::memcpy(kkt, d, S * sizeof(double));
    if (obj) std::memcpy(obj, d + S, S * sizeof(double));
    if (bound) std::memcpy(bound, d + 2 * S, S * sizeof(double));
    if (x) std::memcpy(x, d + 3 * S, nx * sizeof(double));
    if (status) std::memcpy(status, iv, S * sizeof(int));
    if (iters) std::memcpy(iters, iv + S, S * sizeof(int));
    return 0;
}

int phg_solve(phg_handle* h, int32_t w_on, int32_t prox_on, const phg_opts* o) {
    if (!h || !h->loaded) return fail("phg_solve: no batch loaded");
    if (!o) return fail("phg_solve: opts is NULL");
    if (o->check_every <= 0 || o->max_iter <= 0) return fail("phg_solve: bad iteration options");
    CK(hipSetDevice(h->device));
    if (sched_flush(h)) return -1;
    PdhgArgs a{};
    a.S = h->S; a.n = h->n; a.m = h->m; a.nnz = h->nnz; a.N = h->N; a.n_pad = h->n_pad;
    a.lay = h->lay;
    a.vals = h->vals; a.c = h->c; a.cl = h->cl; a.cu = h->cu; a.rl = h->rl; a.ru = h->ru;
    a.dc = h->dc; a.dr = h->dr; a.eta = h->eta; a.obj_off = h->obj_off; a.bnorm = h->bnorm;
    a.W = h->W; a.rho = h->rho; a.xbar = h->xbar; a.xidx = h->xidx; a.fixed = h->fixed;
    a.root_only = h->ph.root_only;
    a.rho_k = h->ph.rho_k;
    a.Z = h->Z; a.Psm = h->Psm; a.smooth_on = h->smooth_on;
    // warm start from the front copy, results into the back copy (swapped after the launch);
    // unscaled x / y are not stored by the solve (materialize_outputs derives them on demand)
    a.xs_in = h->xs; a.ys_in = h->ys; a.omega_in = h->omega;
    a.xs = h->back.xs; a.ys = h->back.ys; a.omega = h->back.omega;
    a.x_out = nullptr; a.y_out = nullptr; a.xN = h->back.xN; a.obj = h->back.obj; a.bound = h->back.bound;
    a.kkt = h->back.kkt; a.iters = h->back.iters; a.status = h->back.status;
    a.order = (o->schedule && h->have_order) ? h->order : nullptr;
    a.iters_acc = h->iters_acc;
    a.w_on = w_on; a.prox_on = prox_on; a.fix_nonants = o->fix_nonants; a.fix_tol = o->fix_tol > 0 ? o->fix_tol : 0.0;
    a.row_fixed = h->row_fixed;
    a.warm = o->warm_start;
    a.max_iter = o->max_iter; a.check_every = o->check_every; a.eps = o->eps_rel; a.sense = h->sense;
    a.beta_suf = o->beta_sufficient > 0 ? o->beta_sufficient : 0.2;
    a.beta_nec = o->beta_necessary > 0 ? o->beta_necessary : 0.8;
    a.beta_art = o->beta_artificial > 0 ? o->beta_artificial : 0.25;
    a.theta = o->primal_weight_theta > 0 && o->primal_weight_theta <= 1 ? o->primal_weight_theta : theta_default(h->n);
    if (h->local_variant >= 0 || h->mfma_variant >= 0) a.check_every = (a.check_every + 1) & ~1;   // 2 iterations per trip
    if (timing_event(h, 0, 0)) return -1;
    a.loc = h->loc;
    a.blk = h->blk;
    a.wv = h->wv;
    a.mf = h->mf;
    a.st = h->st;
    a.gate = o->skip_if_conv_below > 0 ? h->gate : nullptr;
    a.gate_below = o->skip_if_conv_below;
    a.queue = h->persist ? h->queue : nullptr;
    a.avg_every = h->avg_every;
    a.bd = h->bd;
    a.gap_const = h->gap_const;
    a.sum_stride = h->sum_stride;
    {   // PHG_WATCH_SCEN (diagnostic): a scenario whose every PDHG check is printed (the lane-local
        // kernel's PROF instantiation, with PHG_LOCAL_PROF; the MFMA kernel's WATCH instantiation)
        const char* ew = std::getenv("PHG_WATCH_SCEN");
        a.watch = ew ? std::atoi(ew) : -1;
    }
    if (h->fold_w_pending) {
        // the prologue's x = xs dc would not be the caller's xN (xn_external); or the caller did not
        // gate this solve on conv although the head that left the update pending had a convthresh
        // (a final / extension solve after PH converged).  Then the pending W update runs
        // on its own, gated like that head (flush_fold: nothing moves when it found conv below its
        // convthresh -- the reference's break before Update_W, phbase.py:1008-1010), and this solve
        // runs ungated on whatever W that leaves: its outputs are always fresh.  (A head whose
        // convthresh is <= 0 can never have found conv below it -- conv >= 0 -- so its update is
        // unconditional and stays folded into this solve.)
        const bool ungated = !a.gate && h->fold_thr > 0.0;
        if (!fold_active(h) || h->xn_external || ungated) {
            if (flush_fold(h)) return -1;
        } else {
            a.fold_w = 1;   // (gated by the caller, or the head had no convthresh)
            a.W_rw = h->W;
            a.conv_s = h->conv_s;
            a.fold_st = h->fold_st;
            a.status_in = h->status;   // front: the solve whose x the update uses
            h->fold_w_pending = false;
            h->fold_conv_pending = true;
        }
    }
    // the PH update of the pipelined iteration at the end of this launch (ph_tail.h): asked for by
    // phg_set_tail, on a gated prox-QP solve of the lane-local layout that applies a folded update
    // (its per-scenario partials are the convergence metric the tail reduces); PHG_TAIL=0: never
    h->tp.mode = 0;
    {
        static const bool tail_off = [] { const char* e = std::getenv("PHG_TAIL"); return e && std::atoi(e) == 0; }();
        const int mode = h->tail_req;
        h->tail_req = 0;
        // (P <= 128: the metric's per-rank values fit the wave's LDS; every variant's LDS holds the
        // 1 024 doubles of a segment's staging array)
        if (mode && !tail_off && h->local_variant >= 0 && a.fold_w && a.gate && !o->fix_nonants && !a.prof &&
            h->ph.P <= 128 && pdhg_local_lds_bytes(h->local_variant) >= 1024 * sizeof(double)) {
            if (mode == 1 && !h->xbar_next && dalloc(h, &h->xbar_next, 2 * (size_t)std::max(1, h->N_tot))) return -1;
            TailArgs& t = a.tl;
            t.mode = mode;
            const char* eg = std::getenv("PHG_TAIL_GENERIC");   // (read per launch: tests switch it)
            t.generic = (eg && std::atoi(eg)) ? 1 : 0;
            t.segcnt = h->tail_segcnt;
            t.csegcnt = h->tail_csegcnt;
            t.done = h->tail_done;
            t.scen_seg = h->tail_scen_seg;
            t.scen_cseg = h->tail_scen_cseg;
            t.fin = h->tail_fin;
            t.n_fin = h->tail_nfin;
            // PHG_TAIL_PROF=1 (diagnostic): the final wave's stamps, printed after the launch (syncs)
            static unsigned long long* tprof = nullptr;
            t.prof = nullptr;
            if (const char* e = std::getenv("PHG_TAIL_PROF"); e && std::atoi(e)) {
                if (!tprof) CK(hipMalloc((void**)&tprof, 8 * sizeof(unsigned long long)));
                CK(hipMemsetAsync(tprof, 0, 8 * sizeof(unsigned long long), h->stream));
                t.prof = tprof;
            }
            t.out = h->tail_req_out;
            t.xbar_next = h->xbar_next;
            t.xbar_cur = h->xbar;
            t.thr = h->tail_req_thr;
            t.gate = h->gate;
            t.gate_host = h->gate_host;
            t.ph = h->ph;
            t.ph.xN = a.xN;                 // this solve's nonants (the back copy)
            t.ph.conv_s = h->conv_s;        // ... and its prologue's W-update partials
            t.ph.fold_st = h->fold_st;
            h->tp.mode = mode;
            h->tp.thr = t.thr;
            h->tp.gate_below = a.gate_below;
            h->tp.gated_seq = h->wait_seq;  // the gate this solve is predicated on
            h->tp.out = t.out;
            if (mode == 1) t.seq = (double)(h->tp.seq = ++h->gate_seq);
        }
    }
    if (h->border_layout) {
        // PHG_BORDER_PROF=1 (diagnostic, register-resident variant): wall-clock split of a PDHG
        // iteration per workgroup (pdhg_border.hip), printed to stderr after every launch
        static const bool bprof = [] { const char* e = std::getenv("PHG_BORDER_PROF"); return e && std::atoi(e); }();
        static unsigned long long* pbuf = nullptr;
        static size_t pcap = 0;
        const size_t nwg = (size_t)h->st.slots * h->st.K;
        const bool on = bprof && h->bd.reg;
        const size_t need = nwg * 10 + (size_t)h->S * 4;   // + per scenario {start, end, iterations, splits}
        if (on && pcap < need) {
            if (pbuf) CK(hipFree(pbuf));
            CK(hipMalloc((void**)&pbuf, need * sizeof(unsigned long long)));
            pcap = need;
        }
        if (on) CK(hipMemsetAsync(pbuf, 0, pcap * sizeof(unsigned long long), h->stream));
        a.prof = on ? pbuf : nullptr;
        CK(pdhg_border_launch(a, h->stream));
        // PHG_BORDER_STATS=1 (diagnostic, read every launch): the number of split (suspended and
        // re-queued) solves of the launch, to stderr (synchronises the stream)
        if (h->bd.slice > 0 && std::getenv("PHG_BORDER_STATS")) {
            unsigned tail = 0;
            CK(hipMemcpyAsync(&tail, h->st.ctrl + kCtrlTail, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
            CK(hipStreamSynchronize(h->stream));
            fprintf(stderr, "PHG_BORDER_SPLIT slice %d suspended %u of %d\n", h->bd.slice, tail, h->S);
        }
        if (on) {
            std::vector<unsigned long long> hb(need);
            CK(hipMemcpyAsync(hb.data(), pbuf, hb.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
            CK(hipStreamSynchronize(h->stream));
            double t[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
            double span = 0.0;
            for (size_t w = 0; w < nwg; ++w) {
                double tot = 0.0;
                for (int u = 0; u < 10; ++u) t[u] += (double)hb[w * 10 + u];
                for (int u = 0; u < 8; ++u) tot += (double)hb[w * 10 + u];
                span = std::max(span, tot);
            }
            const double it = std::max(1.0, t[8]);
            fprintf(stderr,
                    "PHG_BORDER_PROF K %d slots %d iters %.0f scen %.0f max_wg_us %.1f us_per_iter: primal %.3f "
                    "publish_dual %.3f hop1 %.3f rowsum_mid %.3f hop2 %.3f link_aty %.3f checks %.3f other %.3f\n",
                    h->st.K, h->st.slots, t[8] / h->st.K, t[9] / h->st.K, span / 100.0, t[0] / 100.0 / it,
                    t[1] / 100.0 / it, t[2] / 100.0 / it, t[3] / 100.0 / it, t[4] / 100.0 / it, t[5] / 100.0 / it,
                    t[6] / 100.0 / it, t[7] / 100.0 / it);
            // per scenario: the launch's first start and last end, the heaviest scenario's start offset,
            // span and time per iteration, and the latest first start
            const unsigned long long* sc = hb.data() + nwg * 10;
            unsigned long long t0 = ~0ull, t1 = 0, late = 0;
            int hv = 0;
            double splits = 0;
            for (int q = 0; q < h->S; ++q) {
                t0 = std::min(t0, sc[q * 4]);
                t1 = std::max(t1, sc[q * 4 + 1]);
                if (sc[q * 4 + 2] > sc[hv * 4 + 2]) hv = q;
                splits += (double)sc[q * 4 + 3];
            }
            for (int q = 0; q < h->S; ++q) late = std::max(late, sc[q * 4] - t0);
            const double hdur = (double)(sc[hv * 4 + 1] - sc[hv * 4]) / 100.0;
            fprintf(stderr,
                    "PHG_BORDER_SCEN span_us %.1f heaviest s%d iters %llu start_us %.1f span_us %.1f us_per_iter %.3f "
                    "latest_start_us %.1f splits %.0f\n",
                    (double)(t1 - t0) / 100.0, hv, sc[hv * 4 + 2], (double)(sc[hv * 4] - t0) / 100.0, hdur,
                    hdur / std::max(1.0, (double)sc[hv * 4 + 2]), (double)late / 100.0, splits);
        }
    }
    else if (h->stream_layout) CK(pdhg_stream_launch(a, h->stream));
    else if (h->mfma_variant >= 0) CK(pdhg_mfma_launch(h->mfma_variant, a, h->stream));
    else if (h->local_variant >= 0) {
        // PHG_LOCAL_PROF=1 (diagnostic): per-wave cycle split of the lane-local kernel, summed over
        // the waves and printed to stderr after every launch (synchronises the stream)
        static const bool lprof = [] { const char* e = std::getenv("PHG_LOCAL_PROF"); return e && std::atoi(e); }();
        static unsigned long long* pbuf = nullptr;
        static size_t pcap = 0;
        const size_t waves = (size_t)a.S;   // >= the grid (G scenarios per wave)
        constexpr size_t PW = 10;            // items per wave (pdhg_local.hip, PROF)
        if (lprof && pcap < waves * PW) {
            if (pbuf) CK(hipFree(pbuf));
            CK(hipMalloc((void**)&pbuf, waves * PW * sizeof(unsigned long long)));
            pcap = waves * PW;
        }
        if (lprof) CK(hipMemsetAsync(pbuf, 0, pcap * sizeof(unsigned long long), h->stream));
        a.prof = lprof ? pbuf : nullptr;
        CK(pdhg_local_launch(o->fix_nonants ? h->local_variant : h->local_variant_free, a, h->stream));
        if (lprof) {
            std::vector<unsigned long long> hb(pcap);
            CK(hipMemcpyAsync(hb.data(), pbuf, pcap * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
            CK(hipStreamSynchronize(h->stream));
            double t[6] = {0, 0, 0, 0, 0, 0};
            for (size_t i = 0; i < pcap; ++i)
                if (i % PW < 6) t[i % PW] += (double)hb[i];
            // placement: waves per SIMD (XCD, SE, SH, CU, SIMD from HW_ID) over the launch
            std::map<unsigned long long, int> per_simd;
            for (size_t w = 0; w * PW + 9 < pcap; ++w)
                if (hb[w * PW + 7] > 0) per_simd[(hb[w * PW + 9] << 16) | (hb[w * PW + 8] & 0xFF30ull)]++;
            int simd_max = 0, simd_multi = 0;
            for (auto& kv : per_simd) { simd_max = std::max(simd_max, kv.second); simd_multi += kv.second > 1; }
            // occupancy timeline from the waves' start / end stamps (100 MHz): the launch span, the mean
            // number of resident waves over it, and the span's last part with fewer than half the
            // peak resident (the tail)
            std::vector<std::pair<unsigned long long, int>> ev;
            for (size_t w = 0; w * PW + 7 < pcap; ++w)
                if (hb[w * PW + 7] > hb[w * PW + 6] && hb[w * PW + 6] > 0) {
                    ev.push_back({hb[w * PW + 6], +1});
                    ev.push_back({hb[w * PW + 7], -1});
                }
            std::sort(ev.begin(), ev.end());
            double span = 0, area = 0, tail = 0;
            int peak = 0;
            if (!ev.empty()) {
                int cur = 0;
                for (auto& e : ev) peak = std::max(peak, cur += e.second);
                cur = 0;
                unsigned long long prev = ev[0].first, tail0 = 0;
                for (auto& e : ev) {
                    area += (double)cur * (double)(e.first - prev);
                    const int before = cur;
                    cur += e.second;
                    if (before * 2 >= peak && cur * 2 < peak) tail0 = e.first;   // last drop below half
                    if (cur * 2 >= peak) tail0 = 0;
                    prev = e.first;
                }
                span = (double)(ev.back().first - ev[0].first);
                tail = tail0 ? (double)(ev.back().first - tail0) : 0.0;
            }
            fprintf(stderr,
                    "PHG_LOCAL_PROF iter_cycles %.6e check_cycles %.6e load_cycles %.6e kkt_cycles %.6e restart_cycles %.6e "
                    "checks %.0f span_us %.2f mean_resident %.1f peak_resident %d tail_below_half_us %.2f "
                    "simds_used %zu simds_with_2plus_waves %d max_waves_per_simd %d\n",
                    t[0], t[1], t[2], t[3], t[4], t[5], span / 100.0, span > 0 ? area / span : 0.0, peak, tail / 100.0,
                    per_simd.size(), simd_multi, simd_max);
        }
    }
    else if (h->block_variant >= 0) CK(pdhg_block_launch(h->block_variant, a, h->stream));
    else if (h->wave_variant >= 0) CK(pdhg_wave_launch(h->wave_variant, a, h->stream));
    else CK(pdhg_launch(h->variant, a, h->stream));
    if (timing_event(h, 0, 1)) return -1;
    if (a.tl.mode && a.tl.prof) {
        unsigned long long st[8];
        CK(hipMemcpyAsync(st, a.tl.prof, sizeof st, hipMemcpyDeviceToHost, h->stream));
        CK(hipStreamSynchronize(h->stream));
        auto us = [&](int i, int j) { return st[i] && st[j] ? ((double)st[j] - (double)st[i]) / 100.0 : -1.0; };
        fprintf(stderr, "PHG_TAIL_PROF final wave: its epilogue -> final start %.2f us, final %.2f us\n", us(0, 1),
                us(1, 2));
    }
    h->xn_external = false;
    if (o->safe_bound && !o->fix_nonants) {   // bound.hip: certificates whatever the statuses
        if (!h->sb.Y) {
            if (dalloc(h, &h->sb.Y, (size_t)h->S * h->m)) return -1;
            if (dalloc(h, &h->sb.R, (size_t)h->S * h->n)) return -1;
        }
        if (h->sb_stale && implied_bounds_upload(h)) return -1;
        SafeBoundArgs sb = h->sb;
        sb.all = o->safe_bound >= 2 ? 1 : 0;
        CK(safe_bound_launch(a, sb, h->stream));
    }
    swap_state(h);
    ++h->swaps;
    if (o->schedule && (h->solves % sched_every() == 0 || !h->have_order)) {
        h->sched_pending = true;
        h->sched_src = h->iters;   // (this solve's counts: the front copy after the swap)
        h->sched_unit = a.check_every > 0 ? a.check_every : 1;
    }
    ++h->solves;
    return 0;
}

int phg_node_sums(phg_handle* h, double* dev_nodesum) {
    if (!h || !h->loaded) return fail("phg_node_sums: no batch loaded");
    CK(hipSetDevice(h->device));
    if (h->tp.mode == 2) {
        const bool ran = tail_ran(h) && dev_nodesum == h->tp.out && !h->fold_w_pending;
        h->tp.mode = 0;
        if (ran) {   // the last solve's tail left the node sums and its partials in that buffer
            h->fold_conv_pending = false;
            return 0;
        }
    }
    if (h->fold_w_pending && flush_fold(h)) return -1;   // x changes only by a solve: keep W in step
    if (!h->t_open && timing_event(h, 1, 0)) return -1;
    h->t_open = (h->timing_mask & 2) != 0;
    if (timing_event(h, 2, 0)) return -1;
    PhArgs a = h->ph;
    // a folded update's conv partials ride along into the packed buffer's partials region
    a.fold_conv = h->fold_conv_pending ? 1 : 0;
    a.conv_s = h->conv_s;
    a.fold_st = h->fold_st;
    CK(node_sums_launch(a, dev_nodesum ? dev_nodesum : h->nodesum, h->stream));
    h->fold_conv_pending = false;
    if (carry_flushed_partials(h, dev_nodesum ? dev_nodesum + 2 * (size_t)h->N_tot : nullptr)) return -1;
    if (timing_event(h, 2, 1)) return -1;
    return 0;
}

int phg_apply_xbar(phg_handle* h, const double* dev_nodesum, double* dev_convpart) {
    if (!h || !h->loaded) return fail("phg_apply_xbar: no batch loaded");
    CK(hipSetDevice(h->device));
    if (flush_fold(h)) return -1;
    PhArgs a = h->ph;
    h->gate_fused = dev_convpart == nullptr;   // one GPU: the last workgroup finishes conv too
    if (h->gate_fused) {
        a.gate = h->gate;
        a.gate_host = h->gate_host;
        a.gate_seq = (double)(h->wait_seq = ++h->gate_seq);
    }
    if (!h->t_open && timing_event(h, 1, 0)) return -1;
    if (timing_event(h, 3, 0)) return -1;
    CK(w_update_launch(a, dev_nodesum ? dev_nodesum : h->nodesum,
                       dev_convpart ? dev_convpart : h->convpart, h->stream));
    if (timing_event(h, 3, 1)) return -1;
    if (timing_event(h, 1, 1)) return -1;
    h->t_open = false;
    return 0;
}

int phg_ph_head(phg_handle* h, double* dev_packed, double convthresh, int32_t first) {
    if (!h || !h->loaded) return fail("phg_ph_head: no batch loaded");
    CK(hipSetDevice(h->device));
    PhArgs a = h->ph;
    a.gate = h->gate;
    a.gate_host = h->gate_host;
    a.gate_seq = (double)(h->wait_seq = ++h->gate_seq);
    if (!h->t_open && timing_event(h, 1, 0)) return -1;
    if (timing_event(h, 3, 0)) return -1;
    if (fold_active(h)) {
        // folded: xbar only; W += rho (x - xbar) and its partials in the next solve's prologue
        if (flush_fold(h)) return -1;
        CK(xbar_head_launch(a, dev_packed ? dev_packed : h->packed, convthresh, first, h->stream));
        h->fold_w_pending = true;
        h->fold_thr = first ? -INFINITY : convthresh;
    } else {
        CK(ph_head_launch(a, dev_packed ? dev_packed : h->packed, convthresh, first, h->stream));
    }
    if (timing_event(h, 3, 1)) return -1;
    if (timing_event(h, 1, 1)) return -1;
    h->t_open = false;
    h->gate_fused = false;
    return 0;
}

int phg_ph_step(phg_handle* h, double convthresh, int32_t first, int32_t* out_fused) {
    if (!h || !h->loaded) return fail("phg_ph_step: no batch loaded");
    if (h->tp.mode == 1) {
        const bool ran = tail_ran(h) && !first && convthresh == h->tp.thr && !h->fold_w_pending;
        h->tp.mode = 0;
        if (ran) {   // the last solve's tail did this step: commit its x-bar, take its gate
            if (out_fused) *out_fused = 0;
            std::swap(h->xbar, h->xbar_next);
            h->xsqbar = h->xbar + std::max(1, h->N_tot);
            h->ph.xbar = h->xbar;
            h->ph.xsqbar = h->xsqbar;
            h->fold_conv_pending = false;   // (reduced by the tail into the packed buffer)
            h->fold_w_pending = true;
            h->fold_thr = convthresh;
            h->wait_seq = h->tp.seq;
            h->gate_fused = false;
            return 0;
        }
    }
    const PhArgs& p = h->ph;
    const bool fusable = p.root_only && p.P == 1 && !p.smooth_on && !p.pcv && !h->no_fuse && !fold_active(h);
    if (out_fused) *out_fused = fusable ? 1 : 0;
    // the folded update on one GPU: node sums + x-bar head in one launch (node_sums_kernel HEADX)
    // with phg_node_sums' and phg_ph_head's bookkeeping; PHG_FUSE_HEAD=0: the two launches
    const char* efh = std::getenv("PHG_FUSE_HEAD");   // (read per call: tests switch it)
    const bool fuse_head = !(efh && std::atoi(efh) == 0);
    if (!fusable && fuse_head && fold_active(h)) {
        CK(hipSetDevice(h->device));
        if (h->fold_w_pending && flush_fold(h)) return -1;
        if (!h->t_open && timing_event(h, 1, 0)) return -1;
        if (timing_event(h, 2, 0)) return -1;
        PhArgs a = h->ph;
        a.fold_conv = h->fold_conv_pending ? 1 : 0;
        a.conv_s = h->conv_s;
        a.fold_st = h->fold_st;
        a.gate = h->gate;
        a.gate_host = h->gate_host;
        a.gate_seq = (double)(h->wait_seq = ++h->gate_seq);
        // a due launch schedule rides in this launch as one 256-thread workgroup (up to
        // kSchedFuseMaxS scenarios): farmer 1 250: 0.1018 / 0.1020 vs 0.1027 / 0.1029 ms per PH
        // iteration, 2 500: 0.1367 / 0.1376 vs 0.1378 / 0.1382, 10 000: see kSchedFuseMaxS.
        // PHG_SCHED_FUSE=0 / 1 forces either (A/B)
        const char* esf = std::getenv("PHG_SCHED_FUSE");
        const int sfuse = esf ? std::atoi(esf) : -1;
        if (h->sched_pending && (sfuse == 1 || (sfuse < 0 && h->S <= kSchedFuseMaxS))) {
            a.sched_iters = h->sched_src;
            a.sched_order = h->order;
            a.sched_unit = h->sched_unit;
            h->sched_pending = false;
            h->have_order = true;
        } else if (sched_flush(h)) {
            return -1;
        }
        {   // PHG_HEADX_ONEHOP=0: the ranks meet a second time and the last forms conv (A/B)
            const char* eoh = std::getenv("PHG_HEADX_ONEHOP");
            a.onehop = (eoh && std::atoi(eoh) == 0) ? 0 : 1;
        }
        CK(node_sums_head_launch(a, h->packed, convthresh, first, h->stream));
        h->fold_conv_pending = false;
        if (carry_flushed_partials(h, nullptr)) return -1;
        if (timing_event(h, 2, 1)) return -1;
        if (timing_event(h, 1, 1)) return -1;
        h->t_open = false;
        h->fold_w_pending = true;
        h->fold_thr = first ? -INFINITY : convthresh;
        h->gate_fused = false;
        return 0;
    }
    if (!fusable) {
        if (phg_node_sums(h, nullptr)) return -1;
        return phg_ph_head(h, nullptr, convthresh, first);
    }
    CK(hipSetDevice(h->device));
    PhArgs a = h->ph;
    a.gate = h->gate;
    a.gate_host = h->gate_host;
    a.gate_seq = (double)(h->wait_seq = ++h->gate_seq);
    if (!h->t_open && timing_event(h, 1, 0)) return -1;
    CK(ph_step_launch(a, h->packed, convthresh, first, h->stream));
    if (timing_event(h, 1, 1)) return -1;
    h->t_open = false;
    h->gate_fused = false;
    return 0;
}

int phg_set_col_bounds(phg_handle* h, const double* col_lo, const double* col_hi) {
    if (!h || !h->loaded || !col_lo || !col_hi) return fail("phg_set_col_bounds: no batch loaded / null argument");
    CK(hipSetDevice(h->device));
    const int S = h->S, n = h->n;
    const size_t Sn = (size_t)S * n;
    std::vector<double> L(col_lo, col_lo + Sn), U(col_hi, col_hi + Sn);
    for (size_t f = 0; f < h->fold_col.size(); ++f) {   // rows the presolve folded into these columns
        const int j = h->fold_col[f];
        for (int s = 0; s < S; ++s) {
            L[(size_t)s * n + j] = std::max(L[(size_t)s * n + j], h->fold_lo[f * S + s]);
            U[(size_t)s * n + j] = std::min(U[(size_t)s * n + j], h->fold_hi[f * S + s]);
        }
    }
    for (size_t e = 0; e < Sn; ++e)
        if (!(L[e] <= U[e])) return fail("phg_set_col_bounds: lower bound above upper bound (or NaN)");
    h->tp.mode = 0;
    h->hb.cl = L;
    h->hb.cu = U;
    h->sb_stale = true;
    CK(hipMemcpyAsync(h->cl, L.data(), Sn * sizeof(double), hipMemcpyHostToDevice, h->stream));
    CK(hipMemcpyAsync(h->cu, U.data(), Sn * sizeof(double), hipMemcpyHostToDevice, h->stream));
    CK(scale_cols_launch(h->cl, h->cu, h->dc, (long)Sn, h->stream));   // x = dc xhat: bounds / dc (prep.hip)
    if (h->local_variant >= 0) {
        // the compile-time bound sides of the specialised kernel (BI / BF) must still hold: re-pick
        // the variant of the same shape for the new bounds, then rebuild the lane image (it holds the
        // scaled bounds)
        const phg_batch v = host_view(h);
        LocalPlan plan;
        plan.col_of = h->lp_col_of;
        plan.row_of = h->lp_row_of;
        plan.cpl_row = h->lp_cpl_row;
        const int* sh = h->lshape;
        const unsigned long long bi = local_inf_mask(&v, plan, sh[0], sh[1], sh[2], sh[3]);
        const unsigned long long bf = local_fin_mask(&v, plan, sh[0], sh[1], sh[2], sh[3]);
        const unsigned qm = local_quad_mask(&v, plan, sh[0], sh[1]);
        const char* gen = std::getenv("PHG_LOCAL_GENERIC");
        const int v2 = (gen && std::atoi(gen)) ? h->local_shape_v
                       : pdhg_local_pick_masked(h->local_shape_v, h->local_masks[0], h->local_masks[1], bi, bf, qm);
        const unsigned long long bff = local_fin_mask(&v, plan, sh[0], sh[1], sh[2], sh[3], false);
        const int v2f = (gen && std::atoi(gen)) ? h->local_shape_v
                        : pdhg_local_pick_masked(h->local_shape_v, h->local_masks[0], h->local_masks[1], bi, bff, qm);
        const int ni = pdhg_local_image_items(v2);
        if (ni > h->loc.ni) {
            double* img;
            if (dalloc(h, &img, (size_t)S * ni * sh[0])) return -1;
            h->loc.img = img;
        }
        h->local_variant = v2;
        h->local_variant_free = local_pick_free(v2, v2f);
        h->loc.ni = ni;
        PdhgArgs ia{};
        ia.S = S; ia.n = n; ia.m = h->m; ia.nnz = h->nnz;
        ia.loc = h->loc;
        ia.dc = h->dc; ia.c = h->c; ia.cl = h->cl; ia.cu = h->cu; ia.dr = h->dr; ia.rl = h->rl; ia.ru = h->ru;
        ia.vals = h->vals;
        CK(pdhg_local_image_launch(v2, ia, const_cast<double*>(h->loc.img), const_cast<double*>(h->loc.cimg), h->stream));
    }
    return 0;
}

int phg_set_tail(phg_handle* h, int32_t mode, double convthresh, double* dev_packed) {
    if (!h || !h->loaded) return fail("phg_set_tail: no batch loaded");
    if (mode < 0 || mode > 2) return fail("phg_set_tail: mode must be 0, 1 or 2");
    if (mode == 2 && !dev_packed) return fail("phg_set_tail: mode 2 needs the exchange buffer");
    h->tail_req = mode;
    h->tail_req_thr = convthresh;
    h->tail_req_out = mode == 1 ? h->packed : dev_packed;
    return 0;
}

int phg_tail_info(phg_handle* h, int32_t* out4) {
    if (!h || !h->loaded || !out4) return fail("phg_tail_info: no batch loaded / null argument");
    CK(hipSetDevice(h->device));
    const int ns = h->ph.n_seg, nc = h->ph.n_cseg;
    std::vector<unsigned> c((size_t)ns + nc + 1);
    CK(hipMemcpyAsync(c.data(), h->tail_segcnt, ns * sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
    CK(hipMemcpyAsync(c.data() + ns, h->tail_csegcnt, nc * sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
    CK(hipMemcpyAsync(c.data() + ns + nc, h->tail_done, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
    CK(hipStreamSynchronize(h->stream));
    long armed = 0;
    for (unsigned v : c) armed += v != 0;
    out4[0] = ns + nc;
    out4[1] = h->tail_nfin;
    out4[2] = (int32_t)armed;
    out4[3] = h->tp.mode;
    return 0;
}

int phg_solve_undo(phg_handle* h) {
    if (!h || !h->loaded) return fail("phg_solve_undo: no batch loaded");
    if (h->swaps <= 0) return fail("phg_solve_undo: no solve to undo");
    CK(hipSetDevice(h->device));
    CK(hipStreamSynchronize(h->stream));   // nothing queued may still write the copy being restored
    swap_state(h);
    --h->swaps;
    h->tp.mode = 0;
    return 0;
}

int phg_exchange_layout(phg_handle* h, int32_t* out3) {
    if (!h || !h->loaded || !out3) return fail("phg_exchange_layout: no batch loaded");
    out3[0] = 2 * h->N_tot;                 // node sums
    out3[1] = 2 * h->P + 2;                 // convergence / status partials
    out3[2] = 2 * h->N_tot + 2 * h->P + 3;  // total, incl. the flag
    return 0;
}

int phg_conv_start(phg_handle* h, const double* dev_convpart) {
    if (!h || !h->loaded) return fail("phg_conv_start: no batch loaded");
    CK(hipSetDevice(h->device));
    if (h->fold_conv_pending) {   // the last solve's folded update: its partials first
        CK(fold_conv_launch(h->ph, dev_convpart ? const_cast<double*>(dev_convpart) : h->convpart, h->stream));
        h->fold_conv_pending = false;
        h->gate_fused = false;
    }
    if (!(h->gate_fused && dev_convpart == nullptr))   // after an all-reduce: a small kernel
        CK(conv_gate_launch(dev_convpart ? dev_convpart : h->convpart, h->P, h->gate, h->gate_host,
                            (double)(h->wait_seq = ++h->gate_seq), h->stream));
    h->gate_fused = false;
    return 0;
}

int phg_conv_wait(phg_handle* h, double* host_conv) {
    if (!h || !h->loaded || h->wait_seq == 0) return fail("phg_conv_wait: no phg_conv_start pending");
    // poll the sequence word the kernel stores last (ring slot wait_seq mod 2); every 2^16 polls make
    // sure the stream has not failed (an error would otherwise leave us spinning)
    volatile double* g = h->gate_host + 4 * (h->wait_seq & 1);
    const double want = (double)h->wait_seq;
    for (unsigned long spin = 1; g[3] != want; ++spin) {
        if ((spin & 0xFFFF) == 0) {
            const hipError_t e = hipStreamQuery(h->stream);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(std::string("phg_conv_wait: ") + hipGetErrorString(e));
            if (e == hipSuccess && g[3] != want) return fail("phg_conv_wait: stream idle but no convergence value");
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    *host_conv = g[0];
    h->summary[0] = (int)g[1];
    h->summary[1] = (int)g[2];
    h->last_wait_seq = h->wait_seq;
    h->last_conv = g[0];
    return 0;
}

int phg_conv_finish(phg_handle* h, const double* dev_convpart, double* host_conv) {
    if (phg_conv_start(h, dev_convpart)) return -1;
    return phg_conv_wait(h, host_conv);
}

int phg_set_fold(phg_handle* h, int32_t on, int32_t* active) {
    if (!h) return fail("phg_set_fold: null handle");
    if (h->loaded) {
        CK(hipSetDevice(h->device));
        if (flush_fold(h)) return -1;
    }
    h->fold = on ? 1 : 0;
    if (active) *active = h->loaded && fold_active(h) ? 1 : 0;
    return 0;
}

int phg_fold_partials(phg_handle* h, double* dev_convpart) {
    if (!h || !h->loaded) return fail("phg_fold_partials: no batch loaded");
    CK(hipSetDevice(h->device));
    if (carry_flushed_partials(h, dev_convpart)) return -1;
    if (!h->fold_conv_pending) return 0;
    CK(fold_conv_launch(h->ph, dev_convpart ? dev_convpart : h->convpart, h->stream));
    h->fold_conv_pending = false;
    return 0;
}

int phg_solve_summary(phg_handle* h, int32_t* out2) {
    if (!h || !h->loaded) return fail("phg_solve_summary: no batch loaded");
    out2[0] = h->summary[0];
    out2[1] = h->summary[1];
    return 0;
}

int phg_ph_update(phg_handle* h, double* host_conv) {
    if (phg_node_sums(h, nullptr)) return -1;
    if (phg_apply_xbar(h, nullptr, nullptr)) return -1;
    return phg_conv_finish(h, nullptr, host_conv);
}

int phg_eval_objective(phg_handle* h, int32_t w_on, int32_t prox_on) {
    if (!h || !h->loaded) return fail("phg_eval_objective: no batch loaded");
    if (flush_fold(h)) return -1;
    if (materialize_outputs(h)) return -1;
    CK(hipSetDevice(h->device));
    CK(eval_obj_launch(h->S, h->n, h->N, h->x_out, h->c, h->obj_off, h->nonant_col_d, h->xN, h->W,
                       h->rho, h->xbar, h->xidx, w_on, prox_on, h->sense, h->Z, h->Psm, h->smooth_on, h->eval,
                       h->stream));
    CK(hipStreamSynchronize(h->stream));
    return 0;
}

// ----------------------------------------------------------------------------- RCCL group
// The PH exchange inside the library (SURVEY 8(b) phg_create_group; replaces the MPI Allreduces of
// phbase.py:88-92 and :369 for callers without torch.distributed, e.g. mpi4py ranks that broadcast
// the unique id).  One process per GPU: ncclCommInitRank, not the single-process ncclCommInitAll.
struct phg_group {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

#define NCK(call)                                                                             \
    do {                                                                                      \
        ncclResult_t r_ = (call);                                                             \
        if (r_ != ncclSuccess) return fail(std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");

int phg_group_unique_id(uint8_t* out128) {
    if (!out128) return fail("phg_group_unique_id: null output");
    ncclUniqueId id;
    NCK(ncclGetUniqueId(&id));
    std::memcpy(out128, &id, sizeof id);
    return 0;
}

int phg_create_group(int32_t nranks, int32_t rank, const uint8_t* id128, int32_t device, phg_group** out) {
    if (!out || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return fail("phg_create_group: bad arguments");
    *out = nullptr;
    CK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof id);
    auto* g = new phg_group();
    g->nranks = nranks;
    g->rank = rank;
    g->device = device;
    // non-blocking init, polled with a deadline: a peer that never joins (it failed before its own
    // call) must not leave this rank blocked inside the collective -- on timeout the half-made
    // communicator is aborted and the call fails, so every rank returns and the caller's vote
    // (comm.group_or_host) can fall back.  PHG_GROUP_TIMEOUT seconds (default 300).
    double limit = 300.0;
    if (const char* ev = std::getenv("PHG_GROUP_TIMEOUT")) limit = std::max(1.0, std::atof(ev));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&g->comm, nranks, id, rank, &cfg);
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress || (r == ncclSuccess && g->comm)) {
        ncclResult_t st = ncclInProgress;
        if (ncclCommGetAsyncError(g->comm, &st) != ncclSuccess) { r = ncclSystemError; break; }
        if (st != ncclInProgress) { r = st; break; }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            r = ncclInProgress;
            break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (r != ncclSuccess) {
        if (g->comm) (void)ncclCommAbort(g->comm);
        delete g;
        return fail(r == ncclInProgress
                        ? std::string("phg_create_group: ncclCommInitRankConfig did not complete within ") +
                              std::to_string((int)limit) + " s (a peer never joined?); aborted"
                        : std::string("phg_create_group: ncclCommInitRankConfig: ") + ncclGetErrorString(r));
    }
    *out = g;
    return 0;
}

int phg_group_size(phg_group* g, int32_t* out2) {
    if (!g || !out2) return fail("phg_group_size: null argument");
    // RCCL's own view of the communicator (not the caller's arguments): a bench line that reports
    // these proves the exchange ran over that many ranks
    int cnt = 0, urank = -1;
    NCK(ncclCommCount(g->comm, &cnt));
    NCK(ncclCommUserRank(g->comm, &urank));
    out2[0] = cnt;
    out2[1] = urank;
    return 0;
}

int phg_group_allreduce(phg_group* g, phg_handle* h, double* dev_buf, int64_t count) {
    if (!g || !h || !h->loaded || !dev_buf || count < 0) return fail("phg_group_allreduce: bad arguments");
    if (g->device != h->device) return fail("phg_group_allreduce: the group and the handle are on different devices");
    CK(hipSetDevice(h->device));
    NCK(ncclAllReduce(dev_buf, dev_buf, (size_t)count, ncclDouble, ncclSum, g->comm, h->stream));
    return 0;
}

int phg_ph_exchange(phg_handle* h, phg_group* g) {
    if (!h || !h->loaded) return fail("phg_ph_exchange: no batch loaded");
    int32_t lay[3];
    if (phg_exchange_layout(h, lay)) return -1;
    return phg_group_allreduce(g, h, h->packed, lay[2]);
}

void phg_destroy_group(phg_group* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->comm) (void)ncclCommDestroy(g->comm);
    delete g;
}

int phg_exchange_buffers(phg_handle* h, double** ns, double** cp) {
    if (!h || !h->loaded) return fail("phg_exchange_buffers: no batch loaded");
    if (ns) *ns = h->nodesum;
    if (cp) *cp = h->convpart;
    return 0;
}

int phg_timing_reset(phg_handle* h, int32_t enable) {
    if (!h || !h->loaded) return fail("phg_timing_reset: no batch loaded");
    CK(hipStreamSynchronize(h->stream));
    for (int& c : h->tcount) c = 0;
    h->t_open = false;
    h->timing_mask = enable & 3;
    CK(hipMemsetAsync(h->iters_acc, 0, (size_t)h->S * sizeof(long long), h->stream));
    CK(hipStreamSynchronize(h->stream));
    return 0;
}

int phg_timing(phg_handle* h, int32_t which, double* total_ms, int32_t* launches, int64_t* pdhg_iters) {
    if (!h || !h->loaded) return fail("phg_timing: no batch loaded");
    if (which < 0 || which > 3)
        return fail("phg_timing: which must be 0 (solves), 1 (PH updates), 2 (node sums) or 3 (W updates)");
    CK(hipStreamSynchronize(h->stream));
    double tot = 0.0;
    for (int k = 0; k < h->tcount[which]; ++k) {
        float f = 0.f;
        CK(hipEventElapsedTime(&f, h->tev[which][2 * k], h->tev[which][2 * k + 1]));
        tot += f;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = h->tcount[which];
    if (pdhg_iters) {
        std::vector<long long> acc(h->S);
        CK(hipMemcpy(acc.data(), h->iters_acc, acc.size() * sizeof(long long), hipMemcpyDeviceToHost));
        long long t = 0;
        for (long long v : acc) t += v;
        *pdhg_iters = t;
    }
    return 0;
}


}  // extern "C"
