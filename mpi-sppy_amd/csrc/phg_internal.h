// phg_internal.h -- device-side structures shared by the PH engine's kernels and host API.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace phg {

// Per-lane ownership tables of the wave-per-scenario PDHG kernel.  Built once per batch on the
// host from the SHARED sparsity pattern (see phg_api.hip: build_layout):
//   column j  -> lane j % 64, slot j / 64 ; its CSC entries in that slot (<= KCS)
//   row i     -> lane i % 64, slot i / 64 ; sparse rows keep their CSR entries (<= KRS) in the
//                slot, "dense" rows (> KRS entries) are computed cooperatively by the whole wave
//                (entries dealt round-robin over lanes, <= KD per lane) and reduced with shuffles.
// Padding entries have p = -1 (value 0, index 0).
struct Layout {
    const int* col_of;      // [64*CPL]
    const int* cent_p;      // [64*CPL*KCS]  CSR position of the entry (values are per scenario)
    const int* cent_row;    // [64*CPL*KCS]
    const int* row_of;      // [64*RPL]
    const int* row_dense;   // [64*RPL]      dense-row id or -1
    const int* rent_p;      // [64*RPL*KRS]
    const int* rent_col;    // [64*RPL*KRS]
    const int* dent_p;      // [D*64*KD]
    const int* dent_col;    // [D*64*KD]
    const int* col_nonant;  // [n] nonant index of column j or -1
};

// Lane-local layout of the register-resident PDHG kernel (pdhg_local.hip).  Built on the host by
// partitioning the shared pattern's row/column graph (phg_api.hip: build_local_layout):
//   * "coupling" rows (a few rows linking many blocks, e.g. farmer's total-acreage row) are
//     replicated in every lane of the scenario's lane group and reduced with gsum<LPS>;
//   * every other row lives in the same lane as ALL of its columns, so A x and A^T y for it are
//     plain register FMAs over a dense RPL x CPL block (zero where the pattern has no entry).
struct LocalLayout {
    const int* col_of;      // [LPS*CPL]      column of lane slot, -1 = empty
    const int* row_of;      // [LPS*RPL]      row of lane slot, -1 = empty
    const int* blk_p;       // [LPS*RPL*CPL]  CSR position of entry (row slot, col slot) or -1
    const int* cpl_row;     // [D]            coupling rows (-1 = unused)
    const int* cpl_p;       // [D*LPS*CPL]    CSR position of coupling entry on (lane, col slot) or -1
    // the scenario's constant data in lane order, built once per batch after the preconditioning
    // (pdhg_local.hip local_image_kernel), so the prologue reads it with coalesced, index-free loads:
    // img [S][ni][LPS]: per column slot dc, c (min form, unscaled), scaled lower / upper bound; per row
    // slot 1/dr (0: empty slot), scaled lower / upper bound; the occupied block entries, then the
    // occupied coupling entries (pattern masks MB / MC), scaled.  cimg [S][D][3]: per coupling row
    // 1/dr, scaled lower / upper bound.  slot_kk [LPS*CPL]: nonant index of the slot's column (-1)
    const double* img;
    const double* cimg;
    const int* slot_kk;
    int ni;
};

// Workgroup-per-scenario layout (pdhg_block.hip).  Owner slots: column j -> (slot j / NT,
// thread j % NT), row i likewise.  Row (column) pieces: <= 8 consecutive CSR (CSC) entries; piece p
// -> (slot p / NT, thread p % NT); entry k of a slot-ps piece of thread t sits at
// e = sum_{s < ps} rk[s] NT + k NT + t in the piece-major value / index arrays (coalesced).
struct BlockLayout {
    int n_pad, m_pad;
    const int* col_of;      // [CPL*NT]
    const int* col_pfirst;  // [CPL*NT] first column piece (= LDS partial index) of the column
    const int* col_pcnt;    // [CPL*NT]
    const int* row_of;      // [RPL*NT]
    const int* row_pfirst;  // [RPL*NT]
    const int* row_pcnt;    // [RPL*NT]
    int rk[8], ck[8];       // entries per piece slot (max over the slot's pieces)
    const int* ridx;        // [sum rk NT] column of a row-piece entry (0 on padding)
    const int* cidx;        // [sum ck NT] row of a column-piece entry
    const double* rvals;    // [S or 1][sum rk NT] scaled values, row pieces (0 on padding)
    const double* cvals;    // [S or 1][sum ck NT] scaled values, column pieces
    long vstride_r, vstride_c;   // per-scenario strides (0: one matrix shared by all scenarios)
    // delta form (phg_batch.vals_form): the pieces hold the UNSCALED values -- the constant ones once
    // for all scenarios -- and the kernel applies each scenario's own Ruiz / Pock-Chambolle scaling
    // on the fly (A_hat x = Dr (A (Dc x)): x and y enter the LDS multiplied by dc / dr, the sums leave
    // multiplied by dr / dc; vscale = 1).  Entry row R (the NT entries e = R NT .. R NT + NT - 1 of the
    // piece-major arrays) holding a varying entry reads its values from the scenario's block rdrow[R]
    // of rvd ([S][nd_r NT]; the row's constant entries copied into it too), every other entry row from
    // the shared rvals (vstride_r = 0); -1 = shared
    int vscale;
    int rdrow[32], cdrow[32];
    const double* rvd;
    const double* cvd;
    long dstride_r, dstride_c;
    // unit form (UN variants, delta form only): every constant entry is -1, 0 or +1, so the pieces
    // need no shared values at all -- entry e is the 16-bit code rcode[e] / ccode[e] = the LDS byte
    // address of its x (y) element with the value's sign in bit 0 (padding: the zero slot after y;
    // on the varying entry rows the sign bit is 0 and the values come from rvd / cvd).  The codes and the scenario's nd_r + nd_c varying entry rows are copied into
    // the workgroup's LDS once, so the PDHG iterations read no matrix data from memory.
    int nd_r, nd_c, er, ec;   // varying entry rows; code counts (sum rk NT, sum ck NT)
    const short* rcode;
    const short* ccode;
};

// One-wave-per-scenario shared-matrix layout (pdhg_wave.hip): column at position p of the column
// order (nonants first) -> (slot p / 64, lane p % 64); its <= CE CSC entries; row i -> (slot i / 64,
// lane i % 64); row pieces of <= 8 consecutive CSR entries, piece p -> (slot p / 64, lane p % 64).
// The scaled values (the same in every scenario) are copied into each workgroup's LDS.
struct WaveLayout {
    int n_pad, m_pad;       // per-wave LDS: x [n_pad = CPL*64] by column position, y [m_pad]
    int wave_doubles;       // n_pad + m_pad + PPT * 64
    const int* col_of;      // [CPL*64]
    const int* cidx;        // [CPL*64*CE] row of each column entry (0 on padding, value 0)
    const int* row_of;      // [RPL*64]
    const int* row_pfirst;  // [RPL*64]
    const int* row_pcnt;    // [RPL*64]
    const int* ridx;        // [PPT*8*64] column POSITION of each row-piece entry (0 on padding, value 0)
    const double* rvals;    // [PPT][8][64] scaled values
    const double* cvals;    // [CPL][64][CE]
};

// Shared-matrix MFMA layout (pdhg_mfma.hip): the A operands of v_mfma_f64_16x16x4_f64 for A x
// (fragment (t, u, j): lane l holds A_hat[16 t + (l & 15)][16 u + 4 j + (l >> 4)]) and for A^T y
// (fragment (u, t, j): lane l holds A_hat[16 t + 4 j + (l >> 4)][16 u + (l & 15)]), [fragment][64],
// and which fragments hold a nonzero
struct MfmaLayout {
    const double* frag;     // [2 * 4 TM TN][64]
    unsigned long long nz_ax, nz_aty;
};

// Streaming layout (pdhg_stream.hip): K workgroups per scenario, each owning a row range and a
// column range; the shared pattern in CSR and CSC, the scaled values in both orders, and the
// per-scenario work arrays every PDHG iteration streams
struct StreamLayout {
    int K;
    const int* row_first;   // [K+1]
    const int* col_first;   // [K+1]
    const int* rowptr;      // [m+1]
    const int* colidx;      // [nnz]
    const int* colptr;      // [n+1]
    const int* rowidx;      // [nnz] CSC row indices
    const double* rvals;    // [S or 1][nnz] scaled values, CSR order
    const double* cvals;    // [S or 1][nnz] scaled values, CSC order
    long vstride;           // nnz, or 0 when every scenario has the same matrix
    double *cs, *qs, *lo, *hi, *xsum, *aty, *xr;   // [S*n]
    double *ysum, *axo, *yr;                        // [S*m]
    double* part;           // [slots*K*16] per-workgroup partial sums
    unsigned* ctrl;         // [kCtrlBar + 3*slots] queue head, per-slot barrier counters and mailboxes
    int* err;               // [1] a barrier wait ran past its bound
    int slots;              // groups of K workgroups, each solving queued scenarios one at a time
    int res;                // 1: each workgroup keeps its CSR / CSC slice in LDS (pdhg_stream_lds_bytes)
    int nr_max, nc_max;     // largest per-workgroup nonzero counts (owned rows / owned columns)
    int R_max, C_max;       // largest per-workgroup row / column counts
};
// Bordered block-diagonal layout (pdhg_border.hip): workgroup k of a slot owns a group of column
// blocks and the rows inside them; the NL linking rows are replicated.  Per group, offsets into the
// concatenated arrays below.
struct BorderGroup {
    int c0, nc;          // col_list[c0 .. c0 + nc): owned columns
    int r0, nr;          // row_list[r0 .. r0 + nr): local rows
    int rp0, rz0, nrz;   // rptr[rp0 ..] (nr + 1, local offsets), rcol / rperm[rz0 .. rz0 + nrz)
    int lp0, lz0, nlz;   // lptr[lp0 ..] (NL + 1), lcol / lperm[lz0 .. lz0 + nlz): linking rows on owned columns
    int cp0, cz0, ncz;   // cptr[cp0 ..] (nc + 1), crow / cperm[cz0 .. cz0 + ncz): owned columns (CSC)
    int pad[3];
};
struct BorderLayout {
    int nlink;                       // linking rows (<= 1024: one thread each)
    int nrz_max, nlz_max, ncz_max;   // largest per-group entry counts
    int R_max, C_max;                // largest per-group local-row / column counts
    const BorderGroup* grp;          // [K]
    const int* link_rows;            // [nlink]
    const int *col_list, *row_list;
    const int *rptr, *rcol, *rperm;  // local rows: CSR pointers, columns, positions in the CSR values
    const int *lptr, *lcol, *lperm;  // linking rows restricted to each group
    const int *cptr, *crow, *cperm;  // owned columns: CSC pointers, rows (-(l+1): linking row l), positions
    const int *rcl, *lcl, *crl;      // the same indices as LOCAL positions in the group (register variant)
    double* plink;                   // [slots * 2 * K * nlink * 2] double-buffered linking-row partials
                                     // (register variant: tagged 8-byte granules, two per partial)
    int reg;                         // 0: memory-resident kernel; E = 2: register-resident, E elements per thread
    int xtmp_len;                    // register variant: LDS doubles staging cross-workgroup partials
    // register variant, split solves (pdhg_border.hip): a solve still running after slice x
    // check_every iterations during the queue's first pass is suspended and re-queued (0: off)
    int slice;
    int* requeue;                    // [S] suspended scenarios + 1, in suspension order (zeroed per launch)
    double* susp;                    // [S][8] suspended solves' scalar state
};

constexpr int kCtrlHead = 0;     // StreamLayout::ctrl: queue head
constexpr int kCtrlTail = 1;     //   re-queued (suspended) scenarios so far (bordered split solves)
constexpr int kCtrlDone = 2;     //   scenarios finished (bordered split solves)
constexpr int kCtrlBar = 16;     //   then 2 words per slot (barrier counter), then 1 per slot (mailbox)

struct NodeSeg {           // a contiguous scenario range inside one node (one level)
    int level, node, s0, s1, kofs, klen, seg_first_of_node;
};

struct PhArgs {
    int S, N, N_tot, n_seg, n_cseg, P;
    const double* xN;       // [S*N]
    double* W;              // [S*N]
    const double* rho;      // [S*N]
    const double* rho_k;    // [N] when rho[s*N + k] == rho_k[k] for every scenario (set by phg_set on the
                            // host check; the usual case: defaultPHrho / a per-variable rho_setter), else
                            // null -- the W update then reads N doubles instead of streaming S*N
    const int* xidx;        // [S*N]
    int root_only;          // xidx[s*N + k] == k for all s (two-stage trees): xidx is not read
    const double* pc;       // [S*L]
    const double* pcv;      // [S*N] per-nonant prob coefficients (variable probability) or null
    int L;
    const int* nonant_level;// [N]
    const NodeSeg* seg;     // [n_seg]
    double* segpart;        // [n_seg * 2 * maxk]
    int maxk;
    const int* node_first_seg; // [n_nodes+1] segments of node g: [first[g], first[g+1])
    const int* node_off;    // [n_nodes]
    const int* node_level;  // [n_nodes]
    const int* level_len;   // [L]
    const int* level_kofs;  // [L]
    int n_nodes;
    double* nodesum;        // [2*N_tot]
    double* xbar;           // [N_tot]
    double* xsqbar;         // [N_tot]
    const int* cseg_v;      // [n_cseg] virtual rank of conv segment
    const int* cseg_s0;     // [n_cseg]
    const int* cseg_s1;
    double* csegpart;       // [n_cseg]
    int* csegbad;           // [2*n_cseg] scenarios not optimal / NaN in the last solve
    const int* vr_first;    // [P+1] conv segments of vrank v
    const int* status;      // [S] status of the last solve (may be null)
    double* Z;              // [S*N] smoothing centre (Update_z, phbase.py:329-346), when smooth_on
    const double* beta;     // [S*N]
    int smooth_on;
    unsigned* ticket;       // [3] last-workgroup counters of the two kernels + node_sums' done count
    unsigned* fticket;      // [4] counters of the fused single-GPU step (ph_step_kernel)
    int n_final;            // workgroups sharing node_sums' final reduction (last_k_workgroups)
    // single-GPU PH update: the last w_update workgroup also computes conv into gate (device, read
    // by predicated solves) and gate_host (pinned host memory, read after the handle's event)
    double* gate;
    double* gate_host;
    double gate_seq;
    // folded PH update (PdhgArgs::fold_w): per-scenario sums |x - xbar| and statuses left by the solve
    // prologue; fold_conv: node_sums_kernel also reduces them into the conv partials of the packed
    // exchange buffer (nodesum + 2 N_tot)
    const double* conv_s;
    const int* fold_st;
    int fold_conv;
    // a folded update applied on its own (flush_fold): the head's published conv (gate[0]) and its
    // convthresh -- below it the head left xbar unchanged and W must not move either (the
    // reference's break before Update_W, phbase.py:1008-1010); null: no gate
    const double* skip_gate;
    double skip_below;
    // the launch schedule of the next solve, carried by node_sums_kernel HEADX as one extra
    // workgroup (blockIdx.x == n_seg; schedule.h) when sched_order is set: the last solve's
    // iteration counts (sched_iters) in units of its check interval
    const int* sched_iters;
    int* sched_order;
    int sched_unit;
    // node_sums_kernel HEADX: one hand-off instead of two (every rank forms conv itself)
    int onehop;
};

// The PH update fused into the end of a lane-local solve (ph_tail.h): mode 0 off; 1 one GPU (node
// sums into `out`, convergence partials, gate, next x-bar into xbar_next); 2 multi-GPU (node sums and
// the folded update's convergence partials into the caller's exchange buffer `out`).  Units: the
// node segments (PhArgs::seg) and the conv segments (PhArgs::cseg_*); the wave that completes a unit
// computes its partial, the wave that completes the last unit the final reduction
struct TailArgs {
    int mode;
    int generic;             // 1 (diagnostic / tests, PHG_TAIL_GENERIC=1): segment partials through the
                             // node-sum workgroup's own per-thread loops, one quarter at a time
    unsigned* segcnt;        // [n_seg] scenarios of the node segment counted in (0 between launches)
    unsigned* csegcnt;       // [n_cseg] ... of the conv segment
    unsigned* done;          // [1] units finished
    const int* scen_seg;     // [S*L] node segment of scenario s at level l
    const int* scen_cseg;    // [S] conv segment of scenario s
    const int* fin;          // [4 n_fin] final slots (int4) {element, first segment, terms | stride T << 16, position}
    int n_fin;
    unsigned long long* prof;   // diagnostic (PHG_TAIL_PROF): [3] s_memrealtime stamps, or null
    double* out;             // [2 N_tot node sums | 2P+2 partials | flag]
    double* xbar_next;       // mode 1: [2 N_tot] the next x-bar / x-sq-bar (the current ones if conv < thr)
    const double* xbar_cur;  // mode 1: [2 N_tot]
    double thr;              // mode 1: convthresh
    double seq;              // mode 1: gate sequence number (gate_host slot seq mod 2)
    double* gate;            // mode 1: [3] device gate
    double* gate_host;       // mode 1: [2][4] pinned host ring
    PhArgs ph;               // node segments, conv segments, probabilities, xN / conv_s / fold_st of this solve
};

struct PdhgArgs {
    int S, n, m, nnz, N, n_pad;
    Layout lay;
    LocalLayout loc;
    BlockLayout blk;
    WaveLayout wv;
    MfmaLayout mf;
    StreamLayout st;
    BorderLayout bd;
    // scenario data (scaled where noted)
    const double* vals;     // [S*nnz] scaled values
    const double* c;        // [S*n]   min-form objective, UNscaled
    const double* cl;       // [S*n]   scaled column bounds
    const double* cu;
    const double* rl;       // [S*m]   scaled row bounds
    const double* ru;
    const double* dc;       // [S*n]   column scaling (x = dc * xhat)
    const double* dr;       // [S*m]   row scaling    (A_hat = Dr A Dc)
    const double* eta;      // [S]     step size 0.99 / ||A_hat||_2
    const double* obj_off;  // [S]     min-form constant
    const double* bnorm;    // [S]     ||finite bounds||_2 unscaled
    // PH parameters
    const double* W;        // [S*N]
    const double* rho;      // [S*N]
    const double* rho_k;    // [N] when rho[s*N + k] == rho_k[k] for every scenario (set by phg_set on the
                            // host check; the usual case: defaultPHrho / a per-variable rho_setter), else
                            // null -- the W update then reads N doubles instead of streaming S*N
    const double* xbar;     // [N_tot]
    const int*    xidx;     // [S*N]   xbar slot of (s,k)
    int root_only;          // xidx[s*N + k] == k for every s (two-stage): xidx is not read
    const double* fixed;    // [S*N]
    const double* Z;        // [S*N]   smoothing centre z (smoothed PH, phbase.py:641-760)
    const double* Psm;      // [S*N]   smoothing weight p
    int smooth_on;
    // state (scaled), persists across solves for warm starts: read from the *_in copy, written
    // to the other (the handle's double-buffered solve state, phg_api.hip SolveState)
    const double* xs_in;    // [S*n]
    const double* ys_in;    // [S*m]
    const double* omega_in; // [S]
    double* xs;             // [S*n]
    double* ys;             // [S*m]
    double* omega;          // [S]
    // diagnostic (PHG_LOCAL_PROF, lane-local kernel only): per wave [8] {iteration cycles, check
    // cycles, load cycles, KKT cycles, restart-block cycles, checks}; PHG_BORDER_PROF, the bordered
    // register-resident kernel: per workgroup [10] (pdhg_border.hip); null = off
    unsigned long long* prof;
    int watch;              // with prof (lane-local kernel): scenario whose every check is printed (PHG_WATCH_SCEN), -1 none
    // outputs
    double* x_out;          // [S*n] unscaled, or null: left to phg_get / eval (xs * dc, see unscale_launch)
    double* y_out;          // [S*m] unscaled, or null (ys * dr)
    double* xN;             // [S*N]
    double* obj;            // [S] model sense
    double* bound;          // [S] model sense
    double* kkt;            // [S]
    int*    iters;          // [S]
    int*    status;         // [S]
    const int* order;       // [S] launch order (scenario of work item i), or nullptr = identity
    long long* iters_acc;   // [S] PDHG iterations accumulated over solves (phg_timing_reset zeroes)
    int w_on, prox_on, fix_nonants, warm, max_iter, check_every;
    double fix_tol;                        // fixed nonants: box of half-width fix_tol max(1, |v|)
    const unsigned char* row_fixed;        // [m] 1: every column of the row is a nonant
    double eps, sense;
    double beta_suf, beta_nec, beta_art;   // restart rule
    double theta;                          // primal weight smoothing (1: no smoothing)
    // predicated solve: when gate != nullptr and gate[0] (the convergence metric computed on the
    // device by phg_conv_start) < gate_below, the launch is a no-op -- PH's "break before
    // solve_loop when conv < convthresh" decided on the device, so the host can enqueue the solve
    // before it has read conv back
    const double* gate;
    double gate_below;
    // work queue of the persistent lane-local kernel ([0] next item, [1] waves done; both 0
    // between launches), or nullptr: one work item per lane group
    unsigned* queue;
    int avg_every;          // lane-local kernel: the average iterate's KKT at every avg_every-th check (1: all)
    // 1: the relative gap is taken on the subproblem's whole objective, constant included
    // (obj_off + the prox constant rho/2 ||xbar||^2), as PDLP counts an objective offset:
    //     |p - d| <= eps (1 + |p + K| + |d + K|)
    // -- without K the test is relative to |p|, |d| of the constant-free objective, which the prox
    // term inflates to ~rho/2 ||xbar||^2 (hydro: 1e4 against objectives of order 1); 0: the
    // constant-free form (PHG_GAP_RAW=1, A/B runs)
    int gap_const;
    // lane-local kernel: the average iterate's running sums take every sum_stride-th PDHG iterate
    // (2, the only form compiled since the end of round 4; informational)
    int sum_stride;
    // folded PH update (phg_ph_head with the fold on, include/phg.h): the prologue first applies
    // Update_W of the x it warm-starts from -- W += rho (x - xbar), x = xs_in dc, the bits the last
    // epilogue stored as xN -- writing W in place (W_rw), the scenario's sum |x - xbar| (conv_s) and
    // the status of the solve that produced x (status_in -> fold_st), then solves with the new W
    int fold_w;
    double* W_rw;           // [S*N] = W
    double* conv_s;         // [S]
    int* fold_st;           // [S]
    const int* status_in;   // [S] statuses of the solve being warm-started from (front copy)
    // the PH update of the pipelined iteration at the end of the launch (lane-local layout; ph_tail.h)
    TailArgs tl;
};

// The kernel argument block in the kernarg segment (constant address space: scalar loads).  Cold code
// (prologues, epilogues, checks) reads its pointers through kargs() at the use site -- the laundered
// pointer keeps the compiler from hoisting those loads out of the work loop and holding dozens of
// pointers in SGPRs across it (round 3's lane-local kernel spilled 167 SGPRs to VGPR lanes and
// restored them with ~900 v_readlane in its prologue)
typedef const __attribute__((address_space(4))) PdhgArgs* KP;
__device__ __forceinline__ KP kargs() {
    KP p = (KP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

// The convergence gate for the host: three values, then the sequence number `seq` the host polls,
// into slot seq mod 2 of the fine-grained pinned ring gh[2][4].  Every store is a system-scope
// relaxed store (write-through to host memory: sc0 sc1), and the values are drained (s_waitcnt
// vmcnt(0)) before seq is stored -- so seq never overtakes them, without the system-scope release
// (__threadfence_system / a release store: a write-back of the whole XCD L2, several microseconds
// after a solve has dirtied megabytes of it).  Called by one lane.
__device__ __forceinline__ void publish_host_gate(double* gh_ring, double v0, double v1, double v2, double seq) {
    double* gh = gh_ring + 4 * ((long long)seq & 1);
    __hip_atomic_store(&gh[0], v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&gh[1], v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&gh[2], v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&gh[3], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// relative-gap denominator of the termination test (PdhgArgs::gap_const): K = the objective constant.
// The last term is the round-off floor of the gap itself: p and d are sums of terms of their own
// magnitude, so when the constant nearly cancels them (hydro's prox constant: |p + K| ~ 0.06 against
// |p| ~ 1e4) the gap of an exact floating-point fixed point of the iteration (residuals ~1e-15) can
// sit at ~1e-13 |p| -- above eps (1 + |p + K| + |d + K|) at eps 1e-9, so the solve never stopped (round
// 6: 4 of 20 000 hydro prox-QPs ran to the 2e5 cap at theta 0.5, gap 1.35e-9 against a 1.12e-9
// threshold); a gap within 1e-3 eps (|p| + |d|) is as far as the arithmetic can resolve it
__device__ __forceinline__ double gap_den(double p, double d, double K) {
    return 1.0 + fabs(p + K) + fabs(d + K) + 1e-3 * (fabs(p) + fabs(d));
}

// Safe per-scenario dual bound after a solve (bound.hip, phg_opts.safe_bound): the shared pattern in
// CSR and CSC, the column bounds with every infinite side replaced by one implied by the rows (raw,
// built once per batch on the host: phg_api.hip implied_bounds), the columns that keep an infinite
// side in some scenario (the repair candidates), and per-scenario scratch for the duals / reduced costs
struct SafeBoundArgs {
    const int *rowptr, *colidx;          // [m+1], [nnz]
    const int *colptr, *rowidx, *csc_p;  // [n+1], [nnz] row of CSC entry, [nnz] its CSR position
    const double *ilo, *ihi;             // [S*n] unscaled
    const int* free_col;                 // [nf]
    int nf;
    int all;                             // 1: every scenario (phg_opts.safe_bound = 2), else status != 0 only
    double *Y, *R;                       // [S*m], [S*n]
};

struct PrepArgs {
    int S, n, m, nnz, ruiz_iters, power_iters;
    const int* rowptr;      // [m+1]
    const int* colidx;      // [nnz]
    const int* colptr;      // [n+1]  CSC of the shared pattern
    const int* csc_p;       // [nnz]  CSR position of CSC entry
    const int* row_of_p;    // [nnz]
    double* vals;           // [S*nnz] in: raw values, out: scaled values
    double* dc;             // [S*n]
    double* dr;             // [S*m]
    double* cl; double* cu; // [S*n] in raw, out scaled
    double* rl; double* ru; // [S*m] in raw, out scaled
    double* eta;            // [S]
    double* bnorm;          // [S]
    double* scratch;        // [S*(2n+2m)]
};



// PH terms of nonant t = s*N + k in the min-form subproblem objective (phbase.py:670-760):
//   c += w_on W;  prox_on: c -= rho xbar (+ p z), q = rho (+ p), const += rho/2 xbar^2 (+ p/2 z^2)
// (ph_terms_w: with the value of W given -- the folded update's new W)
// kk = the nonant's index in its scenario (t = s N + kk): two-stage batches (root_only) read xbar[kk]
// and, with rho the same in every scenario (rho_k), rho_k[kk] -- no dependent index load, no S*N
// stream for rho
template <class A>
__device__ __forceinline__ int xbar_slot(const A& a, long t, int kk) {
    return a.root_only ? kk : a.xidx[t];
}
template <class A>
__device__ __forceinline__ double rho_of(const A& a, long t, int kk) {
    return a.rho_k ? a.rho_k[kk] : a.rho[t];
}
template <class A>
__device__ __forceinline__ void ph_terms_w(const A& a, long t, int kk, double w, double& cc, double& qq,
                                           double& pc) {
    if (a.w_on) cc += w;
    if (a.prox_on) {
        const double r = rho_of(a, t, kk);
        const double xb = a.xbar[xbar_slot(a, t, kk)];
        cc -= r * xb;
        qq = r;
        pc += 0.5 * r * xb * xb;
        if (a.smooth_on) {
            const double p = a.Psm[t], z = a.Z[t];
            cc -= p * z;
            qq += p;
            pc += 0.5 * p * z * z;
        }
    }
}
template <class A>
__device__ __forceinline__ void ph_terms(const A& a, long t, int kk, double& cc, double& qq, double& pc) {
    ph_terms_w(a, t, kk, a.w_on ? a.W[t] : 0.0, cc, qq, pc);
}

// scaled box of a fixed nonant t (x = d xhat): [v - w, v + w] / d with w = fix_tol max(1, |v|) --
// 0 fixes exactly; a small positive tolerance plays the part of a CPU solver's primal feasibility
// tolerance when a candidate from a first-order solve meets a first-stage row only to ~1e-10
// (phg_opts.fix_tol)
template <class A>
__device__ __forceinline__ void fixed_box(const A& a, long t, double d, double& lo, double& hi) {
    const double v = a.fixed[t];
    const double w = a.fix_tol * fmax(1.0, fabs(v));
    lo = (v - w) / d;
    hi = (v + w) / d;
}

// scaled bounds of row i (b = s*m + i): with the nonants fixed (xhat evaluation), a row all of whose
// columns are nonants is a constant -- a CPU solver's presolve drops it (or declares the candidate
// infeasible when it is violated beyond its feasibility tolerance; the caller checks that on the
// host, cylinders.evaluate_xhat).  Kept as a row with a first-order solver it would be an equality
// between constants that round-off makes infeasible, sending the dual iterates off along the ray.
template <class A>
__device__ __forceinline__ void row_bounds(const A& a, int i, long b, double& lo, double& hi) {
    if (a.fix_nonants && a.row_fixed && a.row_fixed[i]) { lo = -INFINITY; hi = INFINITY; return; }
    lo = a.rl[b];
    hi = a.ru[b];
}

// PDLP primal weight update at a restart: omega <- (dy/dx)^theta omega^(1-theta), from the squared
// primal / dual movements since the last restart (dx2, dy2; unchanged if either is ~0).  theta 1
// and 0.5 are exact square roots; other values go through the fp32 log2 / exp2 units (a heuristic
// step-size balance: fp32 precision is plenty).
__device__ __forceinline__ double primal_weight(double omega, double dx2, double dy2, double theta) {
    if (!(dx2 > 1e-20 && dy2 > 1e-20)) return omega;
    const double r = sqrt(dy2 / dx2);
    if (theta == 1.0) return r;
    if (theta == 0.5) return sqrt(r * omega);
    const float l = (float)theta * __log2f((float)r) + (1.0f - (float)theta) * __log2f((float)omega);
    return (double)exp2f(l);
}

}  // namespace phg
