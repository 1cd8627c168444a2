"""bench.py -- scenario-QP solves/sec of the PH hot path (farmer cm=10, 10k scenarios) on MI355X.

One "step" = one PH iteration over all scenarios: fused xbar / W / convergence update
(phbase.py:976-1000) + one batched prox-QP solve of every scenario (phbase.py:1023-1030), as the
pipelined PHBase.iterk_loop runs it (one packed all-reduce per iteration across GPUs).
Usage: python bench.py [--gpus N] [--steps K] [--warmup W].  With N > 1 and no WORLD_SIZE in the
environment the script starts ``torch.distributed.run --nproc-per-node N`` on itself as a child
process (before anything touches the GPU) and exits with its return code; under
torch.distributed.run each rank drives one GPU over RCCL.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 dense peak: the VALU rate (v_fma_f64, 64 lanes / 4 cycles per SIMD);
                            # v_mfma_f64_16x16x4_f64 (2048 flop / 64 cycles per SIMD) has the same rate
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E peak


DEFAULT_TRAFFIC = os.path.join(ROOT, "profiles", "traffic_r06.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--case", default="farmer", choices=["farmer", "sslp", "netdes", "hydro", "uc"],
                    help="workload: farmer (the BASELINE.json headline, configs[1]), sslp_15_45_10 or "
                         "netdes network-50-30-H-01 LP relaxations (configs[2], configs[4]), a "
                         "non-uniform 3-stage hydro tree (configs[3], SURVEY 8(d) M3), or the synthetic "
                         "UC-shaped LP relaxation (configs[4], SURVEY 8(d) M5)")
    ap.add_argument("--scen", type=int, default=None,
                    help="scenarios PER GPU (weak scaling); default 10000 farmer, 2048 sslp, 1024 netdes, 2000 hydro, 64 uc")
    ap.add_argument("--cm", type=int, default=10)
    ap.add_argument("--instance", default=None,
                    help="sslp / netdes instance (default sslp_15_45_10 / network-50-30-H-01; held out: "
                         "sslp_5_25_50, network-10-20-H-01)")
    ap.add_argument("--rho", type=float, default=None,
                    help="PH default rho (default 1.0; netdes 10000, the reference's netdes_demo.bash:6 "
                         "--default-rho: PH conv < 1e-4 in 33 s there, 4.3e-3 after 60 s at 1.0)")
    ap.add_argument("--uc-rho", default="default", choices=["cost", "default"],
                    help="uc: --rho everywhere (default: the per-PH-iteration numbers of rounds 1-4) or the "
                         "reference UC's cost-based rho setter (examples/uc/uc_funcs.py:112-132, 0.1 x the "
                         "unit's cost at mid output, as uc_cylinders.py passes it): PH converges ~17x further in "
                         "60 s, each early PH iteration's solves ~15x heavier (DESIGN.md (d))")
    ap.add_argument("--eps", type=float, default=None,
                    help="PDHG relative KKT tolerance (default 1e-9; uc 1e-7, where its bounds are within the "
                         "north star's 1e-6 -- at n ~ 2e4 PDHG needs > 2e5 iterations per solve for 1e-9)")
    ap.add_argument("--eps-schedule", default=None,
                    help="conv-keyed PDHG tolerance schedule 'conv:eps,conv:eps,...' (PHBase pdhg_eps_schedule: "
                         "the first pair whose conv the last known convergence metric reaches, never loosening), "
                         "e.g. '1e-2:1e-5,1e-3:1e-6,0:1e-7'; the solver-option mechanism of the reference's Gapper "
                         "(extensions/mipgapper.py:15-60) keyed by conv instead of the iteration")
    ap.add_argument("--conv-iters", type=int, default=20000, help="PH iteration cap for time-to-conv (0: skip)")
    ap.add_argument("--conv-time", type=float, default=120.0,
                    help="wall cap (s) for time-to-conv (PHBase time_limit; not set for farmer, whose "
                         "iteration cap bounds it, so that no per-iteration host collective is added)")
    ap.add_argument("--conv-scen", type=int, default=None,
                    help="scenarios IN TOTAL of the time-to-conv run (default: the per-GPU default of the "
                         "case, i.e. farmer 10k = the BASELINE headline, sharded over the N GPUs: strong "
                         "scaling)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length (0: skip)")
    ap.add_argument("--cpu-conv-scen", type=int, default=8,
                    help="scenarios of the CPU baseline's time-to-conv leg (farmer: PH to conv < 1e-4 on the "
                         "same processes, one or more scenarios each; 0: skip)")
    ap.add_argument("--cpu-conv-time", type=float, default=90.0, help="wall cap (s) of the CPU time-to-conv leg")
    ap.add_argument("--layout", default="auto", choices=["auto", "gather", "local", "block", "mfma", "stream", "border", "wave"],
                    help="PDHG data layout (include/phg.h: phg_set_layout)")
    ap.add_argument("--no-schedule", action="store_true", help="launch scenarios in index order")
    ap.add_argument("--check-every", type=int, default=None,
                    help="PDHG restart/termination check interval (default: by layout, phbase.check_every_default)")
    ap.add_argument("--beta-art", type=float, default=0.0, help="artificial restart fraction (0: default)")
    ap.add_argument("--beta-suf", type=float, default=0.0, help="sufficient-decay restart factor (0: default 0.2)")
    ap.add_argument("--beta-nec", type=float, default=0.0, help="necessary-decay restart factor (0: default 0.8)")
    ap.add_argument("--theta", type=float, default=0.0, help="primal weight smoothing (0: default)")
    ap.add_argument("--keep-omega", default=None, choices=["fresh", "carry", "blend"],
                    help="PDHG primal weight at each solve: fresh estimate, the previous solve's, or "
                         "their geometric mean (default: by layout, phbase.keep_omega_default)")
    ap.add_argument("--no-presolve", action="store_true", help="keep singleton rows as rows")
    ap.add_argument("--traffic-json", default=DEFAULT_TRAFFIC)
    return ap.parse_args()


def pdhg_flops_per_iter(n, m, nnz):
    # A x (2 nnz) + A^T y (2 nnz); primal update per column: c - A^T y, *tau, x -, /(1+tau q)
    # (incl. 1 mul for tau q, 1 add), clamp (2), running sum (1) = 9; dual update per row:
    # 2 Ax+ - Ax (2), *sig (1), y - (1), + sig*l (2), + sig*u (2), max/min (2), add (1),
    # running sums of y and Ax (2) = 13; A^T y running sum per column (1)
    return 4 * nnz + 10 * n + 13 * m


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def _self_launch(args):
    """--gpus N > 1 outside torch.distributed.run: run N ranks of this script as a child process
    (nothing here has touched the GPU or imported torch) and exit with its return code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, env=env)
    sys.exit(r.returncode)


def _cpu_share():
    """CPU cores this job may use on the host: the cgroup quota if there is one, else the
    OMP_NUM_THREADS the box exports as the per-GPU share, else the affinity mask."""
    vis = len(os.sched_getaffinity(0))
    share, why = vis, "sched_getaffinity"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            share, why = max(1, int(float(q) / float(per))), "cgroup cpu.max"
    except Exception:
        pass
    if why == "sched_getaffinity" and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        share, why = int(os.environ["OMP_NUM_THREADS"]), "OMP_NUM_THREADS (the box's per-GPU CPU share)"
    return max(1, min(share, vis)), vis, why


def _case_setup(args, S, farmer, hydro, netdes, sslp, uc=None):
    nodenames = None
    if args.case == "farmer":
        names, creator = farmer.scenario_names_creator(S), farmer.scenario_creator
        ckw = {"crops_multiplier": args.cm, "num_scens": S}
        desc = f"farmer crops_multiplier={args.cm}"
    elif args.case == "sslp":
        inst = args.instance or "sslp_15_45_10"
        names, creator, ckw = sslp.scenario_names_creator(S), sslp.scenario_creator, {"instance": inst}
        desc = f"{inst} LP relaxation"
    elif args.case == "hydro":
        fan = hydro.synthetic_fanouts(S)
        names, creator, ckw = hydro.scenario_names_creator(S), hydro.synthetic_scenario_creator, {"fanouts": fan}
        nodenames = hydro.synthetic_nodenames(fan)
        desc = f"hydro 3-stage non-uniform tree, stage-2 fan-outs {list(fan)}"
    elif args.case == "uc":
        names, creator, ckw = uc.scenario_names_creator(S), uc.scenario_creator, {"num_scens": S}
        desc = "synthetic UC-shaped LP relaxation (85 generators x 48 periods, N = 4080)"
        if args.uc_rho == "cost":
            desc += ", cost-based rho (the reference's uc rho setter)"
    else:
        inst = args.instance or "network-50-30-H-01"
        names, creator, ckw = netdes.scenario_names_creator(S), netdes.scenario_creator, {"num_scens": S, "instance": inst}
        desc = f"netdes {inst} LP relaxation"
    return names, creator, ckw, nodenames, desc


def _ef_fixture(args, S):
    """The committed EF optimum of this instance (tests/golden/make_ef_fixtures.py), or None."""
    if args.case != "farmer":
        return None
    fn = os.path.join(ROOT, "tests", "golden", f"farmer_cm{args.cm}_ef_S{S}.json")
    if not os.path.exists(fn):
        return None
    return json.load(open(fn))


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        _self_launch(args)
    # stdout carries exactly ONE line, the JSON result: RCCL prints a version banner to stdout when
    # a communicator comes up (at the first collective), so from here on fd 1 points at stderr and
    # the JSON goes to a saved copy of the real stdout
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; PHG_DIST_BACKEND=gloo (CPU-staged all-reduces) lets tests put several ranks
    # on one device -- the production path is nccl (= RCCL over xGMI)
    backend = os.environ.get("PHG_DIST_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count()) if backend != "nccl" else local_rank
    torch.cuda.set_device(device)
    comm = None
    # PHG_FORCE_DIST=1 (tests): the multi-GPU code path on ONE rank -- process group, TorchComm and
    # the packed device exchange all-reduced by the backend (nccl = RCCL), which a one-GPU box can
    # otherwise never run (RCCL refuses two ranks on one device)
    force_dist = os.environ.get("PHG_FORCE_DIST", "0") == "1"
    if force_dist and "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())
    if world > 1 or force_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device(f"cuda:{device}"))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    import _pkg
    _pkg.load()
    from mpisppy_amd import _lib
    from mpisppy_amd import cylinders
    from mpisppy_amd.comm import TorchComm
    from mpisppy_amd.examples import farmer, hydro, netdes, sslp, uc
    from mpisppy_amd.ph import PH
    if world > 1 or force_dist:
        comm = TorchComm()
        # the per-iteration exchange through the library's own RCCL communicator (phg_create_group,
        # on the library's stream): measured on one rank, host + exchange 0.026-0.029 vs 0.034-0.035 ms
        # per PH iteration through torch.distributed's, time to conv 1.02 vs 1.07 s (same trajectory).
        # Setup and host-side collectives stay on torch.distributed.  PHG_EXCHANGE=torch: the torch
        # path (and always under gloo, which puts several ranks on one device)
        if backend == "nccl" and os.environ.get("PHG_EXCHANGE", "lib") == "lib":
            from mpisppy_amd.comm import group_or_host
            comm = group_or_host(comm, device, log=lambda s: print(f"[bench] {s}", file=sys.stderr))

    default_scen = {"farmer": 10000, "sslp": 2048, "netdes": 1024, "hydro": 2000, "uc": 64}[args.case]
    if args.scen is None:
        args.scen = default_scen
    if args.eps is None:
        # uc: 1e-7, the tolerance at which its bounds meet the north star's 1e-6 (test_uc_fullsize_at_north_star_accuracy)
        args.eps = 1e-7 if args.case == "uc" else 1e-9
    if args.rho is None:
        args.rho = 10000.0 if args.case == "netdes" else 1.0
    S = args.scen * world
    names, creator, ckw, nodenames, desc = _case_setup(args, S, farmer, hydro, netdes, sslp, uc)
    opts = {"solver_name": "phg", "PHIterLimit": args.warmup + args.steps, "defaultPHrho": args.rho,
            "convthresh": 1e-4, "verbose": False, "display_progress": False, "pdhg_layout": args.layout,
            "pdhg_schedule": not args.no_schedule, "pdhg_check_every": args.check_every,
            "pdhg_beta_artificial": args.beta_art, "pdhg_beta_sufficient": args.beta_suf,
            "pdhg_beta_necessary": args.beta_nec, "pdhg_primal_weight_theta": args.theta, "pdhg_presolve": not args.no_presolve,
            "pdhg_keep_omega": {None: None, "fresh": False, "carry": True, "blend": "blend"}[args.keep_omega],
            "iterk_solver_options": {"pdhg_eps": args.eps}, "iter0_solver_options": {"pdhg_eps": args.eps},
            "pdhg_exchange": force_dist}
    if args.eps_schedule:
        opts["pdhg_eps_schedule"] = [tuple(float(v) for v in pair.split(":")) for pair in args.eps_schedule.split(",")]
        # Iter0 (no metric yet) at the schedule's first tolerance, as a Gapper's key 0 would set it
        opts["iter0_solver_options"] = {"pdhg_eps": opts["pdhg_eps_schedule"][0][1]}
    args.creator_kwargs = ckw
    t_setup = time.perf_counter()
    rho_setter = uc.rho_setter if args.case == "uc" and args.uc_rho == "cost" else None
    ph = PH(dict(opts), names, creator, mpicomm=comm, scenario_creator_kwargs=ckw, all_nodenames=nodenames,
            rho_setter=rho_setter)
    ph.PH_Prep()
    t_iter0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    t_iter0 = time.perf_counter() - t_iter0
    t_setup = time.perf_counter() - t_setup
    eng = ph.engine
    b = eng.batch
    S_loc = eng.S

    ph.current_solver_options = ph.iterk_solver_options
    # the steps are PHBase.iterk_loop's pipelined iterations (update_and_solve): node sums, ONE
    # all-reduce of the packed exchange buffer, the gated W update (phg_ph_head), the batched solve
    k_iter = [0]

    def step():
        k_iter[0] += 1
        return ph.update_and_solve(first=k_iter[0] == 1)

    for _ in range(args.warmup):
        step()
    # timed region: per-launch HIP events and iteration counts are accumulated on the device and
    # read once afterwards (no per-step host synchronisation beyond PH's own conv readback)
    ev_inline = os.environ.get("PHG_BENCH_EVENTS", "1") != "0"
    eng.timing_reset(solves=ev_inline)
    if comm is not None:
        comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        conv = step()
    torch.cuda.synchronize()
    if comm is not None:
        comm.barrier()
    el = time.perf_counter() - t0
    if not ev_inline:   # (A/B of the events' own cost) the solve launches timed over as many further steps
        eng.timing_reset(solves=True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    pdhg_ms, n_solves, pdhg_iters = eng.timing(0)
    assert n_solves == args.steps, n_solves
    # the PH update timed separately (HIP events only on it) over extra pipelined iterations, as the
    # timed loop ran them: node sums (+ the previous folded update's conv segments) and the head --
    # with the fold (include/phg.h phg_fold_partials) the head only forms xbar and the W update runs
    # in the next solve's prologue; then the standalone two-kernel update (node sums + W update,
    # the sequential statements) for its own roofline
    W_saved = eng.get(_lib.F_W)
    fold = eng.set_fold(os.environ.get("PHG_FOLD", "1") != "0")
    # the timed steps ran the PH update in the solve's tail (ph_tail.h) where it applies: measure the
    # update kernels here with separate launches (their own roofline), the tail off
    tail_on = (ph.options.get("pdhg_tail") if ph.options.get("pdhg_tail") is not None else
               os.environ.get("PHG_TAIL", "0") == "1") and eng.layout == "local" and fold
    ph.options["pdhg_tail"] = False
    eng.timing_reset(solves=False, updates=True)
    for _ in range(args.steps):
        step()
    upd_ms, n_upd, _ = eng.timing(1)
    ns_ms, n_ns, _ = eng.timing(2)
    hd_ms, n_hd, _ = eng.timing(3)
    eng.timing_reset(solves=False, updates=True)
    for _ in range(args.steps):
        ph.Compute_Xbar()
        ph.Update_W()
        ph.convergence_diff()
    sa_ms, n_sa, _ = eng.timing(1)
    sa_ns_ms, n_sa_ns, _ = eng.timing(2)
    sa_wu_ms, n_sa_wu, _ = eng.timing(3)
    eng.timing_reset(solves=False, updates=False)
    eng.set(_lib.F_W, W_saved)
    iters_last = eng.get_i32(_lib.I_ITERS)
    max_iters = int(iters_last.max())
    # per-rank balance: PDHG kernel time and iterations of every rank (max-over-ranks sets the step)
    per_rank = {"pdhg_ms_per_step": [pdhg_ms / args.steps], "pdhg_iters_per_scen": [pdhg_iters / args.steps / S_loc]}
    if comm is not None:
        vec = torch.zeros(2 * world, dtype=torch.float64, device="cuda")
        vec[rank] = pdhg_ms / args.steps
        vec[world + rank] = pdhg_iters / args.steps / S_loc
        dist.all_reduce(vec)
        per_rank = {"pdhg_ms_per_step": [round(v, 4) for v in vec[:world].tolist()],
                    "pdhg_iters_per_scen": [round(v, 2) for v in vec[world:].tolist()]}
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tot = torch.tensor([float(pdhg_iters)], dtype=torch.float64, device="cuda")
        dist.all_reduce(tot)
        pdhg_iters_all = int(tot.item())
    else:
        pdhg_iters_all = pdhg_iters
    S_all = S
    value = S_all * args.steps / el
    ms_per_step = el / args.steps * 1e3

    # roofline of the dominant kernel (batched PDHG), per launch, from HIP events on its stream
    # on the problem the solver runs: singleton rows folded into bounds (one nonzero each) by
    # phg_load_batch's presolve are not part of an iteration
    f_it = pdhg_flops_per_iter(b.n, b.m - eng.rows_folded, b.nnz - eng.rows_folded)
    flops_per_launch = f_it * pdhg_iters / args.steps
    avg_launch_s = pdhg_ms / args.steps / 1e3
    achieved_tf = flops_per_launch / avg_launch_s / 1e12
    # SURVEY 8(d)1 streaming bytes per PDHG iteration per scenario: 16 nnz_distinct + 16 n + 16 m
    # + 8 (n [c varies] + m [b varies]); distinct = CSR positions whose value differs across scenarios
    nnz_distinct = int((b.vals != b.vals[0]).any(axis=0).sum()) if b.S > 1 else 0
    c_var = True    # [c varies] is 1 for every PH prox-QP: W and the prox term make each scenario's cost its own
    b_var = bool((b.rl != b.rl[0]).any() or (b.ru != b.ru[0]).any())
    m_run = b.m - eng.rows_folded
    bytes_it = 16 * nnz_distinct + 16 * b.n + 16 * m_run + 8 * (b.n * c_var + m_run * b_var)
    achieved_gbs = bytes_it * pdhg_iters / args.steps / avg_launch_s / 1e9
    traffic = None
    # PMC bytes per launch (tools/traffic_from_pmc.py): only for the case and kernel (layout) they
    # were measured on -- the default file is the headline's (farmer); another case's PMC bytes only
    # when passed explicitly (--traffic-json), since its kernels changed after the round-2 files
    tpath = args.traffic_json if args.case == "farmer" or args.traffic_json != DEFAULT_TRAFFIC else None
    if tpath and os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("layout") == eng.layout and tj.get("case", "farmer") == args.case:
                traffic = tj.get("pdhg_bytes_per_launch")
        except Exception:
            traffic = None
    valu_pmc = None
    vpath = os.path.join(ROOT, "profiles", "r06", "pmc_valu_mix.json")
    if args.case == "farmer" and eng.layout == "local" and S_loc == 10000 and os.path.exists(vpath):
        try:
            vj = json.load(open(vpath))
            im = vj["issue_model"]
            valu_pmc = {"issue_utilisation": round(im["issue_utilisation"], 4),
                        "issue_model": "fp64 wave64 instruction 4 SIMD cycles, 32-bit 2",
                        "fp64_share_of_valu": round(vj["shares_of_valu"]["fp64 (fma/add/mul/trans)"], 4),
                        "fp64_fma_share_of_valu": round(vj["shares_of_valu"]["fp64 fma"], 4),
                        "fp64_share_of_issue_cycles": round(im["fp64_cycles_share"], 4),
                        "valu_per_wave_iteration": round(vj["valu_per_wave_iteration_counted"], 1),
                        "isa_valu_per_pdhg_iteration": vj["isa_per_pdhg_iteration"]["valu"],
                        "file": "profiles/r06/pmc_valu_mix.json"}
        except Exception:
            valu_pmc = None
    # PH update, algorithmic bytes:
    #   8 S N (1 x read + 1 W read + 1 W write + [rho per scenario ? 1 : 0]) + 8 S + 16 N_tot
    # rho is read from an [N] copy when it is the same in every scenario (PhArgs::rho_k), as here
    rho_now = eng.get(_lib.F_RHO).reshape(S_loc, b.N)
    rho_streams = int(not (rho_now == rho_now[0]).all())
    ph_bytes = 8 * S_loc * b.N * (3 + rho_streams) + 8 * S_loc + 16 * b.N_tot
    sa_gbs = ph_bytes / (sa_ms / max(1, n_sa) / 1e3) / 1e9
    # the node-sum pass on its own bytes: x read (8 S N), prob coefficients (8 S L), the folded
    # update's per-scenario partials and statuses (12 S), node sums written (16 N_tot)
    ns_bytes = 8 * S_loc * b.N + 8 * S_loc * b.L + (12 * S_loc if fold else 0) + 16 * b.N_tot
    ns_s = ns_ms / max(1, n_ns) / 1e3
    ns_gbs = ns_bytes / ns_s / 1e9 if n_ns else 0.0
    # the block kernel on a SHARED matrix (sslp) holds its pieces in registers and x / y in LDS: no
    # per-iteration HBM stream exists to price against the HBM roofline, so it is reported like the
    # register-resident kernels (fp64 flops against the fp64 peak), with the PMC-measured HBM rate beside
    # ... and so is the delta form's unit variant (netdes: the whole matrix in LDS as entry codes plus
    # the scenario's varying entry rows, copied once per solve): no matrix bytes in the iteration
    vinfo = eng.values_info() if eng.layout == "block" else None
    unit = bool(vinfo and vinfo.get("unit"))
    valu = eng.layout in ("local", "gather", "wave") or (eng.layout == "block" and (nnz_distinct == 0 or unit))
    # shared-matrix MFMA layout: SURVEY 8(d)2 F = 4 m n flops per scenario per PDHG iteration (A x and
    # A^T y as dense GEMM) and the flops the matrix cores actually execute (16 x 16 x 4 fragments:
    # 2048 flops per 16 scenarios each, the all-zero ones skipped)
    mfma_rf = None
    if eng.layout == "mfma":
        dense = 4 * b.n * m_run
        frag = eng.mfma_fragments()
        exe = 128 * frag
        mfma_rf = {"bound": "mfma", "achieved": round(dense * pdhg_iters / args.steps / avg_launch_s / 1e12, 4),
                   "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                   "frac": round(dense * pdhg_iters / args.steps / avg_launch_s / 1e12 / FP64_PEAK_TFLOPS, 5),
                   "flops_dense_per_pdhg_iter_per_scen": dense, "mfma_fragments_per_pdhg_iter": frag,
                   "mfma_flops_executed_per_pdhg_iter_per_scen": exe,
                   "executed_tflops": round(exe * pdhg_iters / args.steps / avg_launch_s / 1e12, 4),
                   "flops_sparse_per_pdhg_iter_per_scen": f_it,
                   "sparse_tflops": round(achieved_tf, 4)}

    # the lane-local kernel's EXECUTED work beside the fixed formula: the fp64 operations its hot loop
    # issues per PDHG iteration (phg_local_info, pdhg_local.hip local_loop_ops: FMA = 2; the stride-2
    # running sums, the -sigma-scaled bounds, the folded primal step and the compile-time-dropped
    # clamps as compiled; every lane of the scenario's group, padding lanes included; the restart /
    # termination check every check_every iterations is not counted), and whether the launch took the
    # lone-wave build (small shards)
    exe_rf = {}
    if eng.layout == "local":
        li = eng.local_info()
        exe = li["loop_ops_per_lane"] * li["lanes"]
        exe_tf = exe * pdhg_iters / args.steps / avg_launch_s / 1e12
        exe_rf = {"executed_flops_per_pdhg_iter_per_scen": exe, "executed_tflops": round(exe_tf, 4),
                  "frac_executed": round(exe_tf / FP64_PEAK_TFLOPS, 5), "lone_wave_build": li["lone"],
                  "executed_basis": "hot-loop fp64 ops actually issued (FMA = 2) x lanes per scenario; "
                                    "the check's work excluded"}
    out = {
        "metric": "scenario-QP solves/sec (PH iteration: batched prox-QP solve of every scenario + fused xbar/W/conv)",
        "value": round(value, 2),
        "unit": "scenario-QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": {"farmer": "synthetic (farmer generator of examples/farmer/farmer.py, seeded per scenario)",
                 "sslp": "sslp_15_45_10 data (Scenario1-10) + seeded synthetic ClientPresent beyond 10",
                 "netdes": "network-50-30-H-01 data (30 scenarios) + seeded synthetic cost/capacity noise beyond 30",
                 "hydro": "hydro model of examples/hydro/hydro.py, synthetic inflows A2~U[10,90] per node, "
                          "A3~U[40,60] per leaf (default_rng(1134))",
                 "uc": "synthetic UC-shaped LP (examples/uc.py; egret, which the reference's uc needs, is absent): "
                       "seeded generator data, per-scenario demand and unit derates",
                 }[args.case],
        "config": {"workload": f"{desc}, {S} scenarios ({args.scen} per GPU), PH rho={args.rho}, "
                               f"PDHG eps_rel={args.eps}" + (f", eps schedule {args.eps_schedule}" if args.eps_schedule else ""),
                   "scenarios": S, "n": b.n, "m": b.m, "nnz": b.nnz, "nonants": b.N,
                   "parallelism": f"scenario shards over {world} GPU(s), one packed all-reduce per PH iteration"
                       + (" (libphg RCCL group)" if type(comm).__name__ == "PhgGroupComm" else ""),
                   "pdhg_layout": eng.layout, "lanes_per_scenario": eng.lanes_per_scenario,
                   "presolve_rows_folded": eng.rows_folded,
                   # value form the workgroup kernel streams (phg_values_info): per scenario vs one copy
                   "values": vinfo},
        # fp64 VALU-bound kernels (lane-local / gather): flops against the fp64 peak; the streaming
        # block kernel: algorithmic bytes against HBM
        "roofline": (mfma_rf if mfma_rf is not None else
                     {"bound": "valu", "achieved": round(achieved_tf, 4), "peak": FP64_PEAK_TFLOPS,
                      "unit": "TFLOP/s", "frac": round(achieved_tf / FP64_PEAK_TFLOPS, 5)}
                     if valu else
                     {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(achieved_gbs / HBM_PEAK_GBS, 5), "bytes_per_pdhg_iter_per_scen": bytes_it,
                      "nnz_distinct": nnz_distinct, "tflops_fp64": round(achieved_tf, 4),
                      "valu_frac_fp64": round(achieved_tf / FP64_PEAK_TFLOPS, 5)}) | {
                     "traffic": traffic,
                     # VALU issue measured by PMC on the headline kernel (profiles/r06/pmc_valu_mix.json:
                     # class counters priced 4 cycles per fp64 / 2 per 32-bit wave instruction, over all
                     # SIMDs' cycles of the launch), when this is it
                     "valu_issue_pmc": valu_pmc,
                     # measured HBM rate of the same kernel: PMC bytes per launch / launch duration
                     "hbm_measured_GBs": round(traffic / avg_launch_s / 1e9, 2) if traffic else None,
                     "hbm_measured_frac": round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 5) if traffic else None,
                     "kernel": {"local": "pdhg_local_kernel (lane-local, fp64 VALU)",
                                "gather": "pdhg_kernel (wave LDS-gather, fp64 VALU)",
                                "block": ("pdhg_block_kernel (workgroup per scenario, shared matrix: pieces in registers, "
                                          "x / y in LDS)" if nnz_distinct == 0 else
                                          "pdhg_block_kernel (workgroup per scenario, delta value form: the +-1 entries as "
                                          "LDS address codes and the scenario's varying entry rows in LDS)" if unit else
                                          "pdhg_block_kernel (workgroup per scenario, streamed CSR/CSC pieces)"),
                                "mfma": "pdhg_mfma_kernel (shared matrix, v_mfma_f64_16x16x4_f64, 16 scenarios per wave)",
                                "wave": "pdhg_wave_kernel (one wave per scenario, shared matrix once per workgroup in "
                                        "LDS, no workgroup barrier in the iteration)",
                                "stream": f"pdhg_stream_kernel ({eng.workgroups_per_scenario} workgroups per scenario, "
                                          "range split, iterates and values streamed)",
                                "border": (f"pdhg_border_reg_kernel ({eng.workgroups_per_scenario} workgroups per scenario, "
                                           "bordered block-diagonal, owned state in registers, x / y and slices in LDS, "
                                           "linking rows as tagged-granule reduce-scatter + allgather)"
                                           if eng.border_reg else
                                           f"pdhg_border_kernel ({eng.workgroups_per_scenario} workgroups per scenario, "
                                           "bordered block-diagonal, slices in LDS, linking rows exchanged)")}[eng.layout],
                     "flops_per_pdhg_iter_per_scen": f_it,
                     **exe_rf,
                     "pdhg_iters_per_scen_per_step": round(pdhg_iters / args.steps / S_loc, 2),
                     "max_pdhg_iters": max_iters,
                     "avg_launch_ms": round(avg_launch_s * 1e3, 4)},
        # the PH update as the timed steps run it.  Folded (default on the lane-local layout): the
        # node-sum pass and the xbar head are the only launches -- the W update's x and W reads are
        # the next solve's own warm-start / cost loads and its W write happens there too (measured
        # against the unfolded solve by tools/ph_update_sweep.py); the roofline is the node-sum
        # pass on its own bytes.  "standalone": the two-kernel update (node sums + W update) on
        # the SURVEY 8(d)3 bytes.  At farmer size (10k x 30) every launch here is latency-bound.
        "roofline_ph_update": {"bound": "hbm", "achieved": round(ns_gbs, 2), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(ns_gbs / HBM_PEAK_GBS, 5),
                               "kernel": "node_sums_kernel" + (" (+ the folded update's conv segments)" if fold else ""),
                               "bytes_per_launch": ns_bytes,
                               "path": ("folded: node sums + xbar head; W += rho (x - xbar) in the next PDHG "
                                        "prologue" if fold else "node sums + W update (two launches)"),
                               "avg_ms": round(upd_ms / max(1, n_upd), 4),
                               "node_sums_avg_ms": round(ns_ms / max(1, n_ns), 4) if n_ns else None,
                               "head_avg_ms": round(hd_ms / max(1, n_hd), 4) if n_hd else None,
                               "survey_bytes_per_update": ph_bytes, "rho_streams": rho_streams,
                               "timed": "HIP events on the library stream over extra pipelined iterations "
                                        "with separate launches",
                               "in_solve_tail": bool(tail_on),
                               "note": ("the timed steps ran this update at the end of each solve's launch "
                                        "(ph_tail.h): its time is inside avg_launch_ms" if tail_on else None),
                               "standalone": {"kernels": "node_sums_kernel + w_update_kernel",
                                              "avg_ms": round(sa_ms / max(1, n_sa), 4),
                                              "node_sums_avg_ms": round(sa_ns_ms / max(1, n_sa_ns), 4),
                                              "w_update_avg_ms": round(sa_wu_ms / max(1, n_sa_wu), 4),
                                              "bytes_per_update": ph_bytes, "achieved": round(sa_gbs, 2),
                                              "frac": round(sa_gbs / HBM_PEAK_GBS, 5)}},
        "per_rank": per_rank,
        "host_and_exchange_ms_per_step": round(ms_per_step - max(per_rank["pdhg_ms_per_step"]), 4),
        "setup_s": round(t_setup, 3),
        "iter0_s": round(t_iter0, 4),
        "conv_at_end": conv,
    }
    # who carried the exchange: the path, the collective's own rank count (RCCL's
    # ncclCommCount for the library group), every rank's device / PCI bus id, and the per-iteration
    # all-reduce of the packed buffer timed on the device (HIP events on the stream it runs on)
    from mpisppy_amd.comm import SingleComm, rank_report
    out["ranks"] = rank_report(comm if comm is not None else SingleComm(), device)
    if comm is not None and eng.exchange is not None:
        buf = torch.zeros_like(eng.exchange)
        for _ in range(3):
            comm.allreduce_sum_(buf)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n_ar = 50
        e0.record()
        for _ in range(n_ar):
            comm.allreduce_sum_(buf)
        e1.record()
        torch.cuda.synchronize()
        out["ranks"]["allreduce_us_device"] = round(e0.elapsed_time(e1) / n_ar * 1e3, 2)
        out["ranks"]["allreduce_doubles"] = int(buf.numel())
    if rank == 0:
        print("[bench] timed region done", file=sys.stderr, flush=True)
    cpu_in = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        # the CPU baseline solves the same prox-QPs: this step's W and per-scenario x-bar rows
        W_now = eng.get(_lib.F_W).reshape(eng.S, eng.N)
        xb_nodes = eng.get(_lib.F_XBAR)
        xbar_rows = np.stack([np.concatenate([xb_nodes[b.node_off[g]:b.node_off[g] + b.level_len[lv]]
                                              for lv, g in enumerate(b.scen_node[s])]) for s in range(eng.S)])
        cpu_in = (list(ph.local_scenario_names), W_now, xbar_rows)
    ph.engine.close()

    # wall time to PH convergence < 1e-4: the BASELINE headline instance (farmer 10k IN TOTAL,
    # sharded over the N GPUs), fresh run, the same pipelined iterk_loop as the timed steps
    if args.conv_iters > 0:
        S_c = args.conv_scen or default_scen
        if S_c % world:
            S_c -= S_c % world
        names_c, creator_c, ckw_c, nodenames_c, _ = _case_setup(args, S_c, farmer, hydro, netdes, sslp, uc)
        copts = dict(opts, PHIterLimit=args.conv_iters, convthresh=1e-4,
                     time_limit=None if args.case == "farmer" else args.conv_time)
        ph2 = PH(copts, names_c, creator_c, mpicomm=comm, scenario_creator_kwargs=ckw_c, all_nodenames=nodenames_c,
                 rho_setter=rho_setter)
        ph2.PH_Prep()
        torch.cuda.synchronize()
        if comm is not None:
            comm.barrier()
        tc = time.perf_counter()
        tc0 = tc
        conv2, _, tb2 = ph2.ph_main(finalize=False)
        torch.cuda.synchronize()
        tc = time.perf_counter() - tc
        tc_t = torch.tensor([tc], dtype=torch.float64, device="cuda")
        if comm is not None:
            dist.all_reduce(tc_t, op=dist.ReduceOp.MAX)
        tc = float(tc_t.item())
        eobj = ph2.post_loops()          # E[objective] with W and prox on (ph_main's Eobj)
        ttc = {"scenarios": S_c, "seconds": round(tc, 3), "ph_iters": ph2._PHIter, "conv": conv2,
               "converged": bool(conv2 is not None and conv2 < 1e-4),
               "solves_per_s": round(S_c * ph2._PHIter / tc, 1) if tc > 0 else None,
               "scaling": "strong (the same instance at every N)",
               "trivial_bound": tb2, "Eobj": eobj, "cap_iters": args.conv_iters,
               "cap_s": copts["time_limit"]}
        hist = list(getattr(ph2, "conv_history", []))
        if hist:   # the metric along the run (every ~1/20 of it) and the schedule's last tolerance
            step = max(1, len(hist) // 20)
            ttc["conv_trace"] = [[k + 1, float(hist[k])] for k in range(0, len(hist), step)] + [[len(hist), float(hist[-1])]]
        wt = getattr(ph2, "iter_walltimes", [])
        if len(wt) >= 20:
            ttc["seconds_iter0_and_first_20_ph_iters"] = round(wt[19] - tc0, 3)
        if args.eps_schedule:
            ttc["final_pdhg_eps"] = (ph2.current_solver_options or {}).get("pdhg_eps")
        # inner bound of the converged root xbar (every scenario's nonants fixed to it, W / prox off:
        # xhat_eval.py:102-170) and the gaps to the EF optimum of the same instance
        if b.L == 1:
            xhat = ph2.xbars()[: b.N]
            inner = cylinders.evaluate_xhat(ph2, xhat)
            ttc["xhat_inner_bound"] = inner
            ef = _ef_fixture(args, S_c)
            if ef is not None:
                ttc["ef_objective"] = ef["objective"]
                ttc["rel_gap_Eobj_vs_ef"] = abs(eobj - ef["objective"]) / abs(ef["objective"])
                if inner is not None:
                    ttc["rel_gap_inner_vs_ef"] = (inner - ef["objective"]) / abs(ef["objective"])
                ttc["max_abs_xbar_minus_ef_nonants"] = float(np.max(np.abs(xhat - np.array(ef["root_nonants"]))))
        out["time_to_conv"] = ttc
        ph2.engine.close()

    if cpu_in is not None:
        out["cpu_baseline"] = cpu_baseline(args, *cpu_in)
        if out["cpu_baseline"].get("value"):
            out["cpu_baseline"]["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        if args.case == "farmer" and args.cpu_conv_scen > 0:
            cc = cpu_time_to_conv(args)
            out["cpu_baseline"]["time_to_conv"] = cc
            # the headline instance on the CPU path, PROJECTED (not measured): the GPU run's PH iteration
            # count at its S times S solves per PH iteration at the CPU's measured rates
            ttc = out.get("time_to_conv") or {}
            if cc.get("converged") and ttc.get("ph_iters"):
                S_c, it_c = ttc["scenarios"], ttc["ph_iters"]
                proj = {"what": f"PROJECTION: {it_c} PH iterations (the GPU run's count to conv < 1e-4 at S = "
                                f"{S_c}) x {S_c} solves per PH iteration / CPU solves per second",
                        "scenarios": S_c, "ph_iters": it_c}
                if out["cpu_baseline"].get("value"):
                    proj["at_sample_rate_s"] = round(it_c * S_c / out["cpu_baseline"]["value"], 1)
                if cc.get("solves_per_s"):
                    # the conv run's rate per process, scaled to the job's whole CPU share (the sample's
                    # process count): HiGHS's QP solves are much slower over a PH run's later iterations
                    # than at the sample's state
                    rate = cc["solves_per_s"] / cc["processes"] * out["cpu_baseline"].get("cores", cc["processes"])
                    proj["conv_run_rate_scaled_solves_per_s"] = round(rate, 1)
                    proj["at_conv_run_rate_s"] = round(it_c * S_c / rate, 1)
                out["cpu_baseline"]["projected_time_to_conv_s"] = proj.get("at_conv_run_rate_s") or proj.get("at_sample_rate_s")
                out["cpu_baseline"]["projection"] = proj
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if type(comm).__name__ == "PhgGroupComm":
        comm.close()
    if dist.is_initialized():
        dist.destroy_process_group()


def _cpu_worker(payload):
    """Solve scenario prox-QPs with the oracle (HiGHS 1.8, threads=1; the oracle's interior-point
    QP above 1000 columns, where HiGHS's active-set QP takes minutes) for the time budget.  The
    scenario models are built BEFORE the clock starts (the reference builds its Pyomo models once,
    at setup); the worker cycles over its scenarios until the budget is spent, so the sample is
    budget-long whatever the share size."""
    import time as _t
    sys.path.insert(0, ROOT)
    from oracle import highs
    from oracle import models as om
    case, names, kw, W, xbar, rho, budget = payload
    build = {"farmer": om.farmer, "sslp": om.sslp, "netdes": om.netdes, "hydro": om.hydro_tree, "uc": om.uc}[case]
    probs = []
    for k, nm in enumerate(names):
        sc = build(nm, **kw)
        a = sc.arrays()
        cols = np.array(sc.nonant_cols())
        c = a["c"].copy()
        xb = xbar[k]
        c[cols] += W[k] - rho * xb
        q = np.zeros_like(c)
        q[cols] = rho
        probs.append((c, a, q, float(np.sum(rho / 2 * xb * xb))))
    cnt = 0
    t0 = _t.perf_counter()
    while probs:
        for c, a, q, off in probs:
            left = budget - (_t.perf_counter() - t0)
            r = highs.solve(c, a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"], a["col_lo"],
                            a["col_hi"], qdiag=q, offset=off, do_polish=len(c) > 1000, time_limit=left + 1.0)
            if r.status != "Optimal":   # HiGHS stopped at the sample's time limit: not a completed solve
                return cnt, _t.perf_counter() - t0
            cnt += 1
            if _t.perf_counter() - t0 > budget:
                return cnt, _t.perf_counter() - t0
    return cnt, _t.perf_counter() - t0


def cpu_baseline(args, names, W, xbar):
    """The reference's CPU path restated (oracle): one QP solve per scenario, P processes (the CPU
    share of this job, _cpu_share), on the same W / xbar the GPU just used; bounded sample."""
    import multiprocessing as mp
    if args.case == "uc":
        # measured in the build container: HiGHS 1.8's QP solver returns "Unbounded" after 238 s on
        # one UC prox-QP (the LP relaxation alone: 0.38 s), and the oracle's interior-point QP (dense
        # normal equations, m ~ 2e4) does not finish in 15 min -- no CPU solver here completes a sample
        return {"value": None, "kind": "port", "note": "no CPU QP solver in this image completes a UC "
                "prox-QP (HiGHS 1.8 QP: Unbounded after 238 s; oracle IPM: > 15 min); DESIGN.md (d)"}
    try:
        P, visible, why = _cpu_share()
        per = max(1, len(names) // P)
        kw = args.creator_kwargs
        payloads = [(args.case, names[i * per:(i + 1) * per], kw, W[i * per:(i + 1) * per],
                     xbar[i * per:(i + 1) * per], args.rho,
                     args.cpu_seconds) for i in range(P)]
        ctx = mp.get_context("spawn")
        print(f"[bench] cpu baseline: {P} processes, ~{args.cpu_seconds:.0f} s sample", file=sys.stderr, flush=True)
        with ctx.Pool(P) as pool:
            # hard cap: a worker stuck inside one solve must not hold the GPU measurement hostage
            res = pool.map_async(_cpu_worker, payloads).get(timeout=3 * args.cpu_seconds + 90)
        n = sum(r[0] for r in res)
        t = max(r[1] for r in res)      # the sample's wall time (the slowest worker)
        big = W.shape[1] > 0 and args.case == "netdes"
        solver = "oracle interior-point QP (numpy), one process each" if big else "HiGHS 1.8 via scipy, threads=1 each"
        return {"value": round(n / t, 2), "unit": "scenario-QP solves/s", "cores": P, "kind": "port",
                "cores_visible": visible, "cores_source": why,
                "sample": f"{n} {args.case} prox-QPs ({solver}) on {P} processes in {t:.1f} s "
                          f"(budget {args.cpu_seconds:.0f} s; each process cycles over its {per} scenarios, "
                          "models built before the clock), same W/xbar as the GPU step; excludes Pyomo "
                          "model/objective overhead (lower bound on mpi-sppy CPU time)",
                "sample_seconds": round(t, 2),
                "accuracy": "HiGHS 1.8's QP solver stops ~1e-2 (objective units) short of the optimum on "
                            "these prox-QPs (DESIGN.md (c)); the GPU solves to relative KKT 1e-9"}
    except Exception as e:  # the baseline must never sink the GPU measurement
        return {"value": None, "error": repr(e)}


def _cpu_conv_solve(c, a, q, off):
    """One scenario subproblem on the CPU path (HiGHS 1.8 via scipy, threads=1): plain HiGHS first;
    on its occasional "Solve error" on a plainly feasible farmer prox-QP, again with the infinite
    column bounds capped far outside the data (inactive at the solution), then the oracle's
    certify / polish / interior-point chain.  Returns (x, retried)."""
    from oracle import highs
    args = (c, a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"], a["col_lo"])
    r = highs.solve(*args, a["col_hi"], qdiag=q, offset=off, do_polish=False)
    if r.ok:
        return r.x, 0
    cu = np.asarray(a["col_hi"], float)
    fin = np.concatenate([np.asarray(v, float)[np.isfinite(v)] for v in (a["col_lo"], a["col_hi"], a["row_lo"], a["row_hi"])])
    cap = 1e3 * max(1.0, float(np.abs(fin).max()) if fin.size else 1.0)
    r = highs.solve(*args, np.where(np.isfinite(cu), cu, cap), qdiag=q, offset=off, do_polish=False)
    if r.ok and np.all(np.abs(r.x[~np.isfinite(cu)]) < 0.5 * cap):
        return r.x, 1
    r = highs.solve(*args, a["col_hi"], qdiag=q, offset=off, do_polish=True)
    if not r.ok:
        raise RuntimeError(f"CPU path: no solver certified the subproblem ({r.status})")
    return r.x, 2


def _cpu_conv_worker(rank, P, names, kw, rho, thr, max_it, budget, xs_raw, flag_raw, barrier, out_q):
    """One rank of the CPU path's PH (phbase.py:829-1061 restated for a two-stage tree): its slice of
    the scenarios (sputils.py:819-826), Iter0 LPs, then per iteration Compute_Xbar / Update_W /
    convergence_diff from every rank's nonants in shared memory (the Allreduce of phbase.py:88-92,
    369: every rank sums the same array in the same order, so all ranks take the same decisions)
    and the prox-QP solves.  Models are built before the clock, as the reference builds its Pyomo
    models at setup."""
    import time as _t
    sys.path.insert(0, ROOT)
    from oracle import models as om
    from oracle.ph import rank_slices
    try:
        S = len(names)
        mine = rank_slices(S, P)[rank]
        probs, cols, arr, sgs = [], [], [], []
        for k in mine:
            sc = om.farmer(names[k], **kw)
            arr.append(sc.arrays())
            cols.append(np.array(sc.nonant_cols()))
            sgs.append(1.0 if sc.sense == 1 else -1.0)
        N = len(cols[0])
        xs = np.frombuffer(xs_raw, dtype=np.float64).reshape(S, N)
        flag = np.frombuffer(flag_raw, dtype=np.float64)
        p = np.full(S, 1.0 / S)                       # spbase.py:509-526 default probability
        W = np.zeros((len(mine), N))
        retries = 0

        def solve_all(ph_terms, xbar):
            nonlocal retries
            for j, k in enumerate(mine):
                a = arr[j]
                c = sgs[j] * a["c"].copy()
                q, off = None, 0.0
                if ph_terms:                            # phbase.py:670-760, min form
                    c[cols[j]] += W[j] - rho * xbar
                    q = np.zeros_like(c)
                    q[cols[j]] = rho
                    off = float(np.sum(rho / 2.0 * xbar * xbar))
                x, rt = _cpu_conv_solve(c, a, q, off)
                retries += rt > 0
                xs[k] = x[cols[j]]

        barrier.wait()
        t0 = _t.perf_counter()
        solve_all(False, None)                          # Iter0
        if rank == 0:
            flag[0] = float(_t.perf_counter() - t0 > budget)
        barrier.wait()
        it, conv = 0, None
        while True:
            it += 1
            xbar = p @ xs                               # Compute_Xbar (root node), the same sum everywhere
            W += rho * (xs[mine] - xbar)                # Update_W
            # convergence_diff: mean over ranks of each rank's mean |x - xbar|
            conv = float(np.mean([np.abs(xs[sl] - xbar).mean() for sl in rank_slices(S, P)]))
            stop = conv < thr or it > max_it or flag[0] > 0
            barrier.wait()                              # every rank has read xs
            if stop:
                break
            solve_all(True, xbar)
            if rank == 0:
                flag[0] = float(_t.perf_counter() - t0 > budget)
            barrier.wait()
        out_q.put((rank, it, conv, _t.perf_counter() - t0, retries))
    except Exception as e:   # a rank that fails must not strand the others at the barrier
        barrier.abort()
        out_q.put((rank, -1, repr(e), 0.0, 0))


def cpu_time_to_conv(args):
    """The CPU path's wall time to PH conv < 1e-4, MEASURED on a reduced farmer instance (same
    generator and crops_multiplier, args.cpu_conv_scen scenarios) with one process per scenario up to
    the job's CPU share: Iter0 + PH iterations, each rank solving its scenarios with HiGHS."""
    import multiprocessing as mp
    try:
        S = args.cpu_conv_scen
        share, visible, why = _cpu_share()
        P = max(1, min(share, S))
        from mpisppy_amd.examples import farmer
        names = farmer.scenario_names_creator(S)
        kw = {"crops_multiplier": args.cm, "num_scens": S}
        N = 3 * args.cm
        ctx = mp.get_context("spawn")
        xs_raw = ctx.RawArray("d", S * N)
        flag_raw = ctx.RawArray("d", 1)
        barrier = ctx.Barrier(P)
        q = ctx.Queue()
        print(f"[bench] cpu time-to-conv: farmer cm={args.cm}, {S} scenarios on {P} processes", file=sys.stderr, flush=True)
        procs = [ctx.Process(target=_cpu_conv_worker, args=(r, P, names, kw, args.rho, 1e-4, args.conv_iters or 20000,
                                                            args.cpu_conv_time, xs_raw, flag_raw, barrier, q))
                 for r in range(P)]
        for pr in procs:
            pr.start()
        res, t_end = [], time.perf_counter() + args.cpu_conv_time + 300
        import queue as _queue
        while len(res) < P and time.perf_counter() < t_end:
            try:
                res.append(q.get(timeout=5))
            except _queue.Empty:
                if not any(pr.is_alive() for pr in procs) and q.empty():
                    break                                # every rank died without reporting
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.terminate()
        if len(res) < P:
            return {"converged": False, "error": f"{P - len(res)} of {P} CPU ranks did not report"}
        bad = [r for r in res if r[1] < 0]
        if bad:
            return {"converged": False, "error": bad[0][2]}
        r0 = sorted(res)[0]
        it, conv, secs = r0[1], r0[2], max(r[3] for r in res)
        solves = S * it                                  # Iter0 + (it - 1) prox-QP rounds
        return {"scenarios": S, "processes": P, "cores": P, "cores_source": why, "seconds": round(secs, 2),
                "ph_iters": it, "conv": conv, "converged": bool(conv < 1e-4),
                "solves_per_s": round(solves / secs, 1) if secs > 0 else None,
                "retried_solves": int(sum(r[4] for r in res)),
                "kind": "port", "measured": True,
                "what": f"MEASURED: PH to conv < 1e-4 (rho {args.rho}) on farmer cm={args.cm} with {S} scenarios, "
                        f"{P} processes (one rank each, HiGHS 1.8 via scipy threads=1; shared-memory Allreduce), "
                        "Iter0 included, models built before the clock",
                "accuracy": "HiGHS 1.8's QP stops ~1e-2 (objective units) short of the optimum on these prox-QPs; "
                            "the GPU solves to relative KKT 1e-9"}
    except Exception as e:
        return {"converged": False, "error": repr(e)}


if __name__ == "__main__":
    main()
