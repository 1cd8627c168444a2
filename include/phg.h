/*
 * phg.h -- C ABI of the MI355X (gfx950) Progressive Hedging engine (libphg.so).
 *
 * Replaces, for a batch of scenario subproblems held on one GPU:
 *   - the per-scenario external-solver loop     SPOpt.solve_loop / solve_one
 *                                               (mpisppy/spopt.py:250-341, :99-247)
 *   - PHBase._Compute_Xbar                      (mpisppy/phbase.py:32-112)
 *   - PHBase.Update_W                           (mpisppy/phbase.py:301-326)
 *   - PHBase.convergence_diff                   (mpisppy/phbase.py:349-371)
 *   - the per-scenario bound/objective bookkeeping read by Ebound / Eobjective
 *                                               (mpisppy/spopt.py:225-230, :344-422)
 *
 * Conventions
 *   - return 0 on success, < 0 on error; phg_last_error() gives a thread-local message.
 *   - host arrays are caller-owned and copied in; device memory is owned by the handle.
 *   - all work is ordered on one HIP stream (the handle's own, or one given with
 *     phg_set_stream, e.g. torch.cuda.current_stream()); a handle is not thread-safe.
 *   - "dev_*" pointer arguments are DEVICE pointers (e.g. a torch CUDA tensor's data_ptr) used
 *     for the cross-GPU exchange buffers; every other pointer is a host pointer.
 *   - all floating point is IEEE fp64.
 */
#ifndef PHG_H
#define PHG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct phg_handle phg_handle;

/* A batch of S scenario LPs in standard form sharing one sparsity pattern:
 *     min/max c_s^T x  s.t.  row_lo_s <= A_s x <= row_hi_s,  col_lo_s <= x <= col_hi_s
 * plus the scenario-tree index maps (mpisppy/spbase.py:297-395).  Infinite bounds are +-HUGE_VAL.
 * The xbar vector holds one block per non-leaf tree node: node g's block starts at node_off[g]
 * and has level_len[level of g] entries; the xbar slot of nonant k of scenario s is
 *     node_off[scen_node[s*L + nonant_level[k]]] + nonant_pos[k].                           */
typedef struct phg_batch {
    int32_t S, n, m, nnz;
    const int32_t* rowptr;        /* [m+1] CSR row pointers, shared by all scenarios   */
    const int32_t* colidx;        /* [nnz] column indices, sorted within each row      */
    const double*  vals;          /* [S*nnz] values, CSR order, per scenario           */
    const double*  c;             /* [S*n] objective, in the model's own sense         */
    const double*  col_lo;        /* [S*n] */
    const double*  col_hi;        /* [S*n] */
    const double*  row_lo;        /* [S*m] */
    const double*  row_hi;        /* [S*m] */
    const double*  obj_offset;    /* [S] constant objective term (may be NULL)          */
    int32_t sense;                /* +1 minimize, -1 maximize                           */
    /* scenario tree (non-leaf nodes only, as in mpi-sppy) */
    int32_t N;                    /* nonants per scenario                               */
    const int32_t* nonant_col;    /* [N] column of each nonant (same for all scenarios) */
    int32_t L;                    /* non-leaf levels (1 for two-stage)                  */
    const int32_t* nonant_level;  /* [N] */
    const int32_t* nonant_pos;    /* [N] position inside the node's block               */
    const int32_t* level_len;     /* [L] nonants per node at each level                 */
    const int32_t* scen_node;     /* [S*L] global node id of scenario s at level l       */
    int32_t n_nodes;              /* non-leaf nodes in the WHOLE tree (all ranks)        */
    const int32_t* node_off;      /* [n_nodes] */
    int32_t N_tot;                /* length of the xbar vector                          */
    const double*  prob;          /* [S] scenario probabilities                         */
    const double*  prob_coeff;    /* [S*L] p_s / P(node)  (spbase.py:382-395)            */
    /* rank slicing of the reference run whose convergence metric is reproduced
     * (phbase.py:349-371 averages per-rank means): scenario s of this batch is global
     * scenario scen_global0 + s of S_global, sliced over virt_nproc ranks
     * (sputils.py:819-826).                                                                */
    int32_t scen_global0;
    int32_t S_global;
    int32_t virt_nproc;
    /* variable_probability (spbase.py:398-438): [S*N] per-nonant prob coefficients replacing
     * prob_coeff in the node sums; W of a zero-probability nonant is kept at 0 (phbase.py:323-326).
     * NULL when unused.                                                                      */
    const double*  prob_coeff_var;
    /* Value forms ("values: shared [nnz] or per-scenario [S*nnz] or a sparse delta
     * list"; the reference's scenario_creator builds each scenario's model in full, so which
     * coefficients vary is the instance's, e.g. netdes varies only the u_e of its vubs,
     * examples/netdes/netdes.py:39-80):
     *   PHG_VALS_PER_SCENARIO (0; callers that zero the struct): vals is [S*nnz];
     *   PHG_VALS_SHARED       (1): vals is [nnz], one matrix for every scenario;
     *   PHG_VALS_DELTA        (2): vals is [nnz], a shared base; the n_delta CSR positions
     *                             delta_pos[] (strictly increasing) take per-scenario values
     *                             delta_vals[S*n_delta] (scenario-major).
     * Whatever the form, phg_load_batch finds the positions whose value differs between scenarios;
     * when they are few (<= nnz/2) and the workgroup layout is chosen, all scenarios share one
     * scaling and one copy of the constant entries, and the solver streams only the varying ones
     * (PHG_DELTA=0 in the environment: per-scenario scaling and copies, for A/B runs).          */
    int32_t vals_form;
    int32_t n_delta;
    const int32_t* delta_pos;
    const double*  delta_vals;
} phg_batch;
enum { PHG_VALS_PER_SCENARIO = 0, PHG_VALS_SHARED = 1, PHG_VALS_DELTA = 2 };

typedef struct phg_opts {
    double  eps_rel;       /* relative KKT tolerance (PDLP-style), e.g. 1e-9            */
    int32_t max_iter;      /* PDHG iteration limit per scenario                         */
    int32_t check_every;   /* iterations between restart/termination checks (e.g. 64)   */
    int32_t warm_start;    /* bit 0: start from the previous x, y; bit 1: keep its primal weight;
                              bit 2: start from sqrt(previous x fresh) primal weight          */
    int32_t fix_nonants;   /* 1: nonants fixed to the values set by phg_set_fixed (xhat) */
    int32_t schedule;      /* 1: launch scenarios heaviest-first by the previous solve's PDHG
                              iteration counts (device counting sort after each solve)       */
    /* restart rule (PDLP-style; <= 0 selects the default): restart when the KKT error of the
     * candidate drops below beta_sufficient x the last restart's, or below beta_necessary x it
     * while rising, or after beta_artificial x (iterations so far) without a restart          */
    double  beta_sufficient;   /* default 0.2  */
    double  beta_necessary;    /* default 0.8  */
    double  beta_artificial;   /* default 0.25 (tuned on PH prox-QPs; PDLP uses 0.36) */
    /* primal weight smoothing at restarts, omega <- (dy/dx)^theta omega^(1-theta);
     * (0, 1], <= 0 selects the default by subproblem size n (after presolve): 0.8 for
     * n < 2 000, 0.5 for n < 10 000, 0.05 above (PDLP uses 0.5; measured on MI355X, round 3:
     * farmer 0.8 best, netdes 0.5 +8-11 % over 0.8, UC 0.05 7.8x fewer ms per PH iteration)   */
    double  primal_weight_theta;
    /* > 0: the solve is a device-side no-op when the convergence metric of the handle's last
     * phg_conv_start is below this value (PH's "conv < convthresh: stop before solve_loop",
     * phbase.py:1008-1010, decided on the device so the solve can be enqueued before conv is
     * read back); 0: always solve                                                             */
    double  skip_if_conv_below;
    /* fix_nonants: each fixed value v becomes the box [v - w, v + w], w = fix_tol * max(1, |v|)
     * (0: exact).  The reference's xhat evaluation fixes exactly and relies on the CPU solver's
     * primal feasibility tolerance (~1e-6 absolute) when a candidate violates a first-stage row by
     * round-off (an xbar of first-order solves: farmer 10k sums to 5000 + 2e-7 acres); an exactly
     * fixed infeasible box sends PDHG's dual iterates off along the infeasibility ray instead.     */
    double  fix_tol;
    /* 1: after the solve, replace the dual bound (PHG_F_BOUND) of every scenario that did not reach
     * the KKT tolerance (status 1 / 2; the others keep the solve's dual objective) by a bound that is
     * valid whatever the status -- the Lagrangian dual function of the scenario's subproblem at the
     * solve's dual iterate, made feasible: row duals of the wrong sign for an infinite row bound
     * zeroed; columns charged against their bounds, infinite ones replaced by bounds implied by the
     * rows (computed once per batch from the caller's data); reduced-cost infeasibility on a column
     * with no finite bound either way repaired by shrinking the duals of its rows.  -inf (+inf when
     * maximising) only when no finite certificate results.  For the bound consumers of spopt.py:
     * 225-230 (Iter0's trivial bound, spopt.py:377-422 Ebound; the Lagrangian spoke,
     * lagrangian_bounder.py:21-44) at scenarios that stopped at the iteration limit.  Not with
     * fix_nonants.  2: the certificate for EVERY scenario -- the dual objective of a converged solve
     * is accurate to eps (1 + |p| + |d|) on either side of the optimum, as a CPU solver's bound is at
     * its tolerances; at a loose eps (UC runs at 1e-6) that can sit above the optimum by ~1e-6
     * relative, the certificate never does.                                                     */
    int32_t safe_bound;
} phg_opts;

/* solve modes (mpisppy/phbase.py:670-760: W_on / prox_on toggles) */
enum { PHG_W_OFF = 0, PHG_W_ON = 1 };
enum { PHG_PROX_OFF = 0, PHG_PROX_ON = 1 };

/* fields for phg_get / phg_set (host copies) */
enum {
    PHG_F_X = 0,        /* [S*n]  primal solution, unscaled                                 */
    PHG_F_Y = 1,        /* [S*m]  row duals (min-form sign convention: >= 0 at lower bound) */
    PHG_F_XN = 2,       /* [S*N]  nonant values (PH x), unscaled                           */
    PHG_F_W = 3,        /* [S*N]  PH dual weights                                          */
    PHG_F_RHO = 4,      /* [S*N]  PH penalties                                             */
    PHG_F_XBAR = 5,     /* [N_tot] node averages                                           */
    PHG_F_XSQBAR = 6,   /* [N_tot] node averages of x^2                                    */
    PHG_F_OBJ = 7,      /* [S] primal objective of the last solve, model sense, incl. W/prox */
    PHG_F_BOUND = 8,    /* [S] dual (outer) bound of the last solve, model sense           */
    PHG_F_EVAL = 9,     /* [S] objective evaluated by phg_eval_objective                  */
    PHG_F_KKT = 10,     /* [S] final relative KKT error                                    */
    PHG_F_FIXED = 11,   /* [S*N] values nonants are fixed to when opts.fix_nonants         */
    PHG_F_CONV_PART = 12,/* [2*virt_nproc+2] per-virtual-rank (sum |x-xbar|, count), then the
                            status counts of phg_solve_summary                              */
    PHG_F_OMEGA = 13,   /* [S] PDHG primal weight carried between solves                    */
    PHG_F_Z = 14,       /* [S*N] smoothing centre z (smoothed PH)                          */
    PHG_F_SMOOTH_P = 15,/* [S*N] smoothing weight p                                        */
    PHG_F_SMOOTH_BETA = 16,/* [S*N] smoothing step beta                                    */
    PHG_F_WARM = 17     /* phg_copy_from only: src's last solution (scaled x, y and primal weights)
                           as dst's warm start -- e.g. a Lagrangian spoke starting from the hub's
                           prox-QP solution, whose duals are near-optimal for the Lagrangian LP once
                           x is near xbar                                                       */
};
enum {
    PHG_I_ITERS = 0,    /* [S] PDHG iterations of the last solve                           */
    PHG_I_STATUS = 1,   /* [S] 0 optimal (KKT <= eps), 1 iteration limit, 2 numerical error */
    PHG_I_ORDER = 2     /* [S] launch order of the next solve (heaviest first; a due schedule is
                           computed first).  Undefined until the first scheduled solve          */
};

int  phg_create(int device, phg_handle** out);
void phg_destroy(phg_handle* h);
const char* phg_last_error(void);
int  phg_set_stream(phg_handle* h, void* hip_stream);
int  phg_sync(phg_handle* h);

/* PDHG data layout, chosen at phg_load_batch (call before it):
 *   AUTO   : when every scenario has the same constraint matrix and it fits the MFMA tiles
 *            (n, m <= 16: one 16 x 16 tile) densely enough (nnz >= 1/16 of the padded
 *            tile) and the batch holds >= 4096 scenarios (one 16-scenario wave per CU), the
 *            shared-matrix fp64 MFMA layout (pdhg_mfma.hip, 16 scenarios per wave);
 *            else the lane-local register layout (pdhg_local.hip) when the pattern splits into
 *            blocks that fit a lane plus <= a few coupling rows, else the wave LDS-gather layout
 *            (pdhg.hip, n, m <= 256), else the workgroup-per-scenario streaming layout
 *            (pdhg_block.hip, n, m up to 4096), else a multi-workgroup layout (K workgroups per
 *            scenario): the bordered block-diagonal one (pdhg_border.hip: column blocks coupled by
 *            <= 1024 linking rows, slices in LDS, one cross-workgroup exchange per iteration) when
 *            the pattern has that structure, else the range-split one (pdhg_stream.hip, any size)
 *   WAVE   : (on request only) one wavefront per scenario, the matrix once per workgroup in LDS
 *            (pdhg_wave.hip: every scenario the same matrix, columns with <= 2 entries, n <= 1024,
 *            m <= 64; measured slower than BLOCK on sslp)
 *   GATHER / LOCAL / BLOCK / MFMA / STREAM / BORDER / WAVE : that layout or fail (MFMA, WAVE: shared matrix
 *            only; STREAM: the range-split kernel)                                             */
enum { PHG_LAYOUT_AUTO = 0, PHG_LAYOUT_GATHER = 1, PHG_LAYOUT_LOCAL = 2, PHG_LAYOUT_BLOCK = 3,
       PHG_LAYOUT_MFMA = 4, PHG_LAYOUT_STREAM = 5, PHG_LAYOUT_BORDER = 6, PHG_LAYOUT_WAVE = 7 };
int  phg_set_layout(phg_handle* h, int32_t policy);
/* host-only dry run of the lane-local planner (no device needed): out8 = {local shape or -1,
 * lanes per scenario, columns per lane, rows per lane, coupling-row slots, coupling rows used,
 * lanes used, the kernel variant phg_load_batch runs (pattern / infinite-bound specialised)}      */
int  phg_plan(const phg_batch* b, int32_t* out8);

/* singleton-row presolve, on by default (call before phg_load_batch): rows with one nonzero on a
 * non-nonant column become bounds on that column (same LP; PDHG handles bounds exactly).  phg_get /
 * phg_set of PHG_F_Y keep the caller's row numbering; folded rows read back 0.
 * phg_presolve_info: out2 = {rows folded, rows kept}                                          */
int  phg_set_presolve(phg_handle* h, int32_t on);
/* host-only (no device): the column bounds phg_opts.safe_bound uses -- every infinite bound of
 * scenario s that a row implies replaced by that implied bound (bound propagation over the rows,
 * widened against round-off), finite ones unchanged; lo, hi are [S*n]; *n_free (may be NULL) = the
 * columns left with an infinite side in some scenario.  On the batch as given (no presolve).     */
int  phg_implied_bounds(const phg_batch* b, double* lo, double* hi, int32_t* n_free);
int  phg_presolve_info(phg_handle* h, int32_t* out2);
int  phg_load_batch(phg_handle* h, const phg_batch* b);
/* phg_set returns once host_in is copied (to page-locked staging); the device copy is ordered on the
 * handle's stream before everything enqueued after it.  phg_get / phg_get_i32 synchronise.        */
int  phg_set(phg_handle* h, int32_t field, const double* host_in);
int  phg_get(phg_handle* h, int32_t field, double* host_out);
int  phg_get_i32(phg_handle* h, int32_t field, int32_t* host_out);
/* the last solve's per-scenario results in ONE synchronisation (replaces phg_sync + phg_get_i32
 * STATUS / ITERS + phg_get KKT / OBJ / BOUND / X after a solve: what a solver plugin returns per
 * solve, spopt.py:184-231); any pointer may be NULL.  status, iters, kkt, obj, bound: [S]; x: [S*n]  */
int  phg_solve_results(phg_handle* h, int32_t* status, int32_t* iters, double* kkt, double* obj,
                       double* bound, double* x);
/* shared-matrix MFMA layout: out4 = {row tiles, column tiles, 16x4 fragments with a nonzero in
 * A x, in A^T y} (each is one v_mfma_f64_16x16x4_f64 per PDHG iteration per 16 scenarios)       */
int  phg_mfma_info(phg_handle* h, int32_t* out4);
/* value form of the loaded batch (phg_batch.vals_form): out4 = {CSR positions whose value differs
 * between scenarios, 1 if all scenarios share one scaling and one copy of the constant entries (the
 * delta form is in use; 2: its unit form -- every constant entry is +-1 and the kernel holds the
 * matrix in LDS as 16-bit entry codes), matrix values the PDHG kernel reads PER SCENARIO in one
 * A x + A^T y, shared entries in one A x + A^T y} (workgroup layout; the other layouts
 * report {varying, 0, 0, 0})                                                                        */
int  phg_values_info(phg_handle* h, int32_t* out4);
/* lane-local layout: out4 = {variant, lanes per scenario, 1 if the next launch takes the lone-wave
 * build (every wave alone on its SIMD: a grid of at most 4 x CUs waves, PHG_LOCAL_LONE), executed
 * fp64 operations per PDHG iteration per lane of the variant's hot loop x 100 (pdhg_local.hip
 * local_loop_ops; FMA counted as 2)}                                                                  */
int  phg_local_info(phg_handle* h, int32_t* out4);
int  phg_info(phg_handle* h, int32_t* out8);   /* S, n, m, nnz, N, N_tot, kernel variant
                                                  (>= 100: lane-local, >= 200: workgroup,
                                                  >= 300: shared-matrix MFMA, 400 + K:
                                                  range-split streaming, 500 + K / 600 + K:
                                                  bordered block-diagonal, memory- /
                                                  register-resident; K workgroups per
                                                  scenario), lanes (threads) per scenario  */

/* Solve every scenario's subproblem (solve_loop):
 *   min-form  c^T x + w_on * sum_k W_k x_k + prox_on * sum_k rho_k/2 (x_k - xbar_k)^2      */
int  phg_solve(phg_handle* h, int32_t w_on, int32_t prox_on, const phg_opts* opts);

/* PH update, split for an external (RCCL / torch.distributed) all-reduce between steps:
 *   1. phg_node_sums   : dev_nodesum[2*N_tot] <- local sums of prob_coeff*x, prob_coeff*x^2
 *   2. (all-reduce SUM of dev_nodesum across GPUs)
 *   3. phg_apply_xbar  : xbar <- nodesum; W += rho (x - xbar); dev_convpart[2*virt_nproc+2]
 *   4. (all-reduce SUM of dev_convpart[2*virt_nproc + 2] across GPUs)
 *   5. phg_conv_finish : conv = (1/P) sum_v sum_v/count_v
 * phg_ph_update does 1-5 on one GPU (no exchange).                                          */
int  phg_node_sums(phg_handle* h, double* dev_nodesum);
int  phg_apply_xbar(phg_handle* h, const double* dev_nodesum, double* dev_convpart);
int  phg_conv_finish(phg_handle* h, const double* dev_convpart, double* host_conv);
/* phg_conv_finish split in two: phg_conv_start enqueues the conv computation (into the handle's
 * device gate, read by predicated solves) and its copy to the host; phg_conv_wait blocks until
 * that copy has landed -- work enqueued in between (the next solve) keeps the GPU busy         */
int  phg_conv_start(phg_handle* h, const double* dev_convpart);
int  phg_conv_wait(phg_handle* h, double* host_conv);
/* status summary of the solve preceding the last PH update, read back by phg_conv_finish with the
 * convergence partials (dev_convpart[2P], [2P+1]; summed over GPUs by the same all-reduce):
 * out2 = {scenarios not at the KKT tolerance, scenarios with a numerical failure}            */
int  phg_solve_summary(phg_handle* h, int32_t* out2);
int  phg_ph_update(phg_handle* h, double* host_conv);

/* Pipelined PH iteration with ONE exchange per iteration (replaces the two Allreduces of
 * phbase.py:88-92 and :369 inside iterk_loop, phbase.py:976-1035).  The exchange buffer is packed:
 *     dev_packed = [2*N_tot node sums | 2*virt_nproc+2 conv / status partials | 1 flag]
 * (phg_exchange_layout: out3 = {node-sum length, partials length, total}; NULL dev_packed = the
 * handle's own buffer, for one GPU).  One iteration k is
 *     phg_node_sums(h, dev_packed)      local node sums of the current x (the last solve's)
 *     (all-reduce SUM of dev_packed across GPUs: node sums of x_k AND the partials of update k-1)
 *     phg_ph_head(h, dev_packed, thr, k == 1)
 *                                       conv_{k-1} from the partials -> device gate + host word;
 *                                       unless conv_{k-1} < thr: xbar, W += rho (x - xbar), and the
 *                                       partials of update k into dev_packed
 *     phg_solve(..., skip_if_conv_below = thr)   gated on conv_{k-1} as well
 *     phg_conv_wait(h, &conv)           conv_{k-1} (+inf at k = 1: no metric yet)
 * The solve is therefore speculative by one: conv_{k-1} < thr means PH stopped BEFORE solve k-1
 * (phbase.py:1008-1010).  The device has then skipped update k and solve k, and because solves
 * double-buffer their state and a gated solve writes nothing, the state is exactly the one before
 * solve k-1 (x_{k-2}, W_{k-1}, xbar_{k-1}).  After the last iteration, phg_conv_start on the
 * partials gives conv of the last update; if it is below thr, phg_solve_undo restores the state
 * before the last solve.                                                                         */
/* Folded update (lane-local layout without smoothing / variable probability; by default on for
 * batches with S*N >= 1e7 nonant values and off below -- measured slower on farmer 10k, faster at
 * S*N = 1e8; phg_set_fold / PHG_FOLD override): phg_ph_head
 * then only publishes conv_{k-1} and forms xbar_k; the next
 * phg_solve applies W += rho (x - xbar) in its prologue -- it loads x (its warm start) and W (its
 * objective) anyway, so the update's second read of x and its own launch disappear -- and leaves
 * the per-scenario partials of update k on the device.  The next phg_node_sums reduces them into the
 * partials region of the packed buffer it is given (dev_nodesum + 2*N_tot: pass the packed buffer),
 * so the one all-reduce still carries them; after the last pipelined iteration
 * phg_fold_partials(h, dev_convpart) does that reduction alone (before the caller's all-reduce of the
 * partials; phg_conv_start does it itself when nothing is to be all-reduced, dev_convpart NULL).
 * Reading or writing W / xbar, phg_apply_xbar or a second head before a solve apply a pending
 * update first, so the state stays the reference's.                                           */
int  phg_fold_partials(phg_handle* h, double* dev_convpart);
/* fold on / off for this handle (a pending folded update is applied first); *active (may be NULL)
 * = 1 if the loaded batch's solves take the folded update                                      */
int  phg_set_fold(phg_handle* h, int32_t on, int32_t* active);
int  phg_exchange_layout(phg_handle* h, int32_t* out3);
int  phg_ph_head(phg_handle* h, double* dev_packed, double convthresh, int32_t first);
int  phg_solve_undo(phg_handle* h);
/* Fuse the NEXT iteration's PH update into the end of the NEXT phg_solve (one-shot request; the
 * pipelined loop sets it before every solve): mode 1 (one GPU) -- node sums of the solve's x, the
 * convergence metric of the folded W update its prologue applied, the gate and the next x-bar (the
 * current one if conv < convthresh), all of which the following phg_ph_step then takes over instead
 * of launching; mode 2 (exchange) -- node sums and partials into dev_packed, taken over by the
 * following phg_node_sums(h, dev_packed); 0: off.  Only the lane-local layout with the folded
 * update, on a gated solve; otherwise the request is dropped and the separate launches run.
 * Replaces nothing in mpi-sppy by itself: it is the launch schedule of phbase.py:976-1030 on one
 * device.  The tail's sums are the separate launches' bit for bit (ph_tail.h: each node / conv
 * segment reduced by the wave that completes it, the final reduction by the wave that completes the
 * last segment; no wave waits on another).  PHG_TAIL=0 disables it.                                */
int  phg_set_tail(phg_handle* h, int32_t mode, double convthresh, double* dev_packed);
/* Diagnostic (synchronises): out4 = {tail units (node + conv segments), final-reduction slots,
 * unit / done counters not at zero (0 between launches: each is re-armed by the wave that
 * completes it), the mode of the last solve's tail (0: none)}                                    */
int  phg_tail_info(phg_handle* h, int32_t* out4);
/* New column bounds of the loaded batch ([S*n] each, the caller's units; +-inf allowed) without a
 * reload: intersected again with the rows the presolve folded into bounds, scaled on the device,
 * the lane-local kernel re-picked for the new bound sides and its lane image rebuilt; the safe-bound
 * pass's implied bounds are recomputed at the next safe-bound solve.  What the reference's
 * _fix_nonants / _restore_nonants (spopt.py:590-640) change on a persistent solver (update_var). */
int  phg_set_col_bounds(phg_handle* h, const double* col_lo, const double* col_hi);
/* One GPU (nothing to exchange): phg_node_sums + phg_ph_head on the handle's own buffer.  With
 * PHG_FUSE=1 and a batch that allows it (two-stage tree, one virtual rank, no smoothing, no variable
 * probability) as ONE launch (the node-sum pass, then the W update by the last workgroups, x
 * streamed once; the same bits as the two launches) -- measured slower than the two launches on
 * farmer 10k, so off by default.  out_fused (may be NULL) = 1 if the fused kernel ran.           */
int  phg_ph_step(phg_handle* h, double convthresh, int32_t first, int32_t* out_fused);

/* smoothed PH (phbase.py:329-346, 641-760): while on, every prox-on solve adds
 * p/2 (x_k - z_k)^2 per nonant and phg_apply_xbar also does Update_z: z += beta (x - z)        */
int  phg_set_smoothing(phg_handle* h, int32_t on);

/* per-scenario objective with the CURRENT W/xbar/rho (pyo.value(objfct), spopt.py:365) */
int  phg_eval_objective(phg_handle* h, int32_t w_on, int32_t prox_on);


/* Cylinders on one GPU (hub.py:462-616 send_ws / send_nonants, spoke.py; here device-to-device,
 * ordered after src's queued work by an event, enqueued on dst's stream):
 *   phg_copy_from : dst.field <- src.field (W for a Lagrangian spoke, phbase.py:397-413; PHG_F_WARM:
 *                   src's last solution becomes dst's warm start)
 *   phg_fix_from  : dst.fixed[s, :] <- src.xN[scen, :] for all s (xhat candidate = scenario scen's
 *                   nonants, xhatshufflelooper_bounder.py; two-stage batches)
 *   phg_query     : *idle = 1 when everything queued on h's stream has finished (non-blocking)  */
int  phg_copy_from(phg_handle* dst, phg_handle* src, int32_t field);
int  phg_fix_from(phg_handle* dst, phg_handle* src, int32_t scen);
int  phg_query(phg_handle* h, int32_t* idle);

/* launch timing without per-launch synchronisation: phg_timing_reset clears the counters and
 * selects what gets HIP events (enable bit 0: solves, bit 1: PH updates; 0 = none, the
 * production default);
 * phg_timing sums the HIP-event durations of every solve (which = 0), PH update (which = 1: from the
 * node sums' begin to the W update's end), node-sum launch (2) or W-update / head launch (3)
 * launched since, and the PDHG iterations of all scenarios over those solves              */
int  phg_timing_reset(phg_handle* h, int32_t enable);
int  phg_timing(phg_handle* h, int32_t which, double* total_ms, int32_t* launches, int64_t* pdhg_iters);

/* device pointers into the handle's own packed exchange buffer: its node sums (2*N_tot doubles)
 * and its conv / status partials (2*virt_nproc+2 doubles, followed by the flag)                */
int  phg_exchange_buffers(phg_handle* h, double** dev_nodesum, double** dev_convpart);

/* RCCL group: the cross-GPU exchange inside the library (SURVEY 8(b) phg_create_group), for callers
 * without torch.distributed -- e.g. the reference's mpi4py ranks: rank 0 calls phg_group_unique_id
 * and MPI_Bcast's the 128 bytes, then every rank calls phg_create_group with its own device (one
 * process per GPU: ncclCommInitRank; collective over the nranks processes).  Replaces the MPI
 * Allreduces of phbase.py:88-92 (node sums) and :369 (convergence) for the pipelined iteration:
 *     phg_node_sums(h, NULL); phg_ph_exchange(h, g); phg_ph_head(h, NULL, thr, first); phg_solve(...)
 *   phg_group_allreduce : in-place SUM of count doubles at dev_buf, on h's stream (h on g's device)
 *   phg_ph_exchange     : phg_group_allreduce of h's own packed exchange buffer
 *   phg_group_size      : out2 = {ncclCommCount, ncclCommUserRank} of the communicator          */
typedef struct phg_group phg_group;
int  phg_group_unique_id(uint8_t* out128);
int  phg_create_group(int32_t nranks, int32_t rank, const uint8_t* id128, int32_t device, phg_group** out);
int  phg_group_size(phg_group* g, int32_t* out2);
int  phg_group_allreduce(phg_group* g, phg_handle* h, double* dev_buf, int64_t count);
int  phg_ph_exchange(phg_handle* h, phg_group* g);
void phg_destroy_group(phg_group* g);

#ifdef __cplusplus
}
#endif
#endif /* PHG_H */
