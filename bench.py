"""Benchmark: ADMM iterations/s of the DDPCA-ADMM solve loop on a synthetic DEHW-shaped mesh.

Workload (BASELINE.json configs[4]): 8 subdomains of 1.23M DOF each
(9.8M DOF), 4 worm/wheel groups -- each a frictional contact (mu = 0.2) between a worm block and
a wheel block -- glued into two chains along x, 6 multigrid levels per subdomain, and M3's
interface density: 7.9M integration points (0.80 per DOF, DEHW's 3.37M ip / 4.18M DOF) -- contact
faces integrated over 4 x 4 polygons each, glued faces over 2 x 2 (what CSEARCH's intersection
yields against a slave surface mesh 4x / 2x finer, as DEHW's adaptively refined contact bands).  One ADMM
iteration = every subdomain's MGPIS PCG solve (1e-14 recursive residual, x0 = 0, as
MGPIS::CG_SOLV) + the interface-eliminated coarse-space correction (muscSett = 2, doleMcsc = 1:
DEHW's own setting, DEHW.h:2222, 2239) + the interface step + MONITOR.  The global problem is fixed and its subdomains
are spread over the ranks (strong scaling); N = 1 runs all 8 on one MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints one JSON line.  `roofline` is the fine-level SELL-BSR3 SpMV kernel (the dominant
kernel family, one launch covers every owned subdomain), timed by HIP events around its launch in
the eager first PCG iteration of every batched solve, on the solve stream;
`cpu_baseline` is the CPU port (oracle/cpu_admm.py: SGS-faithful MGPIS + the interface step) pricing
one full ADMM iteration of the same workload at the device run's final state.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
VALUE_LAYOUT = "fp64-pairs, col16"  # SELL layout of the fine Krylov operator (device_mgpis.hip)


def parse():
    H = importlib.import_module("ddpca-admm_amd").HEADLINE_OPTIONS  # pinned by tests/test_headline_gpu.py
    M = importlib.import_module("ddpca-admm_amd").HEADLINE_MUSC
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    W = importlib.import_module("ddpca-admm_amd").HEADLINE_WORKLOAD  # the same parity tests pin it
    ap.add_argument("--groups", type=int, default=W["groups"], help="worm/wheel groups (2 subdomains each)")
    ap.add_argument("--nx", type=int, default=W["nx"])
    ap.add_argument("--ny", type=int, default=W["ny"])
    ap.add_argument("--nz", type=int, default=W["nz"])
    ap.add_argument("--gl", type=int, default=W["gl"], help="uniform refinements (levels = gl + 1)")
    ap.add_argument("--fric", type=float, default=W["fric"])
    ap.add_argument("--ip-contact", type=int, default=W["ip_contact"],
                    help="contact faces integrated over 2^k x 2^k polygons (k = 2: M3's 0.8 ip per DOF with --ip-glued 1)")
    ap.add_argument("--ip-glued", type=int, default=W["ip_glued"], help="the same for the glued faces")
    # defaults: the fastest configuration of the round-1 sweep (profiles/r01_sweep.txt)
    ap.add_argument("--smoother", type=int, default=None, help="0 point Jacobi, 1 block Jacobi, 2 Chebyshev, "
                    "3 multicolour block Gauss-Seidel on the fine level (block Jacobi below, --nu sweeps), 4 the same as colour SSOR; default: "
                    "headline_options(subdomains per rank) -- 3 with nu 2 above 4 subdomains per rank, else 1 with nu 2")
    ap.add_argument("--nu", type=int, default=None)
    ap.add_argument("--omega-scale", type=float, default=-H["omega"],
                    help="Jacobi damping = scale / lambda_max(M^-1 K) per level (profiles/r01_sweep_omega.txt)")
    ap.add_argument("--iters-per-graph", type=int, default=H["iters_per_graph"])
    ap.add_argument("--warm-start", type=int, default=H["warm_start"],
                    help="1: each subdomain PCG starts from its previous solution (same 1e-14 stop rule)")
    ap.add_argument("--precond-fp32", type=int, default=H["precond_fp32"],
                    help="1: V-cycle level operators stored in fp32; 2: and the finest levels' V-cycle copies in block-exponent fp16; "
                         "3: in block-scaled int8 instead; 4: as 3, the fine colour sweeps gathering an fp32 copy of "
                         "the iterate (arithmetic, Krylov operator and stop rule fp64)")
    ap.add_argument("--table-mode", type=int, default=H["table_mode"],
                    help="1: keep one copy of bit-identical operator rows (pays on regular meshes only; the "
                         "synthetic box mesh is far more regular than DEHW's curved one, so the headline keeps 0)")
    ap.add_argument("--musc", type=int, default=M["muscSett"],
                    help="muscSett: 2 = interface-eliminated coarse space every ADMM iteration (DEHW.h:2222), 0 = none")
    ap.add_argument("--dole", type=int, default=M["doleMcsc"], help="doleMcsc: coarse-space level of every subdomain (DEHW.h:2239)")
    ap.add_argument("--coarse-level", type=int, default=H["coarse_level"],
                    help="V-cycle level of the exact dense coarse solve (-1: auto, 0: the reference's)")
    ap.add_argument("--mesh", choices=["headline", "general"], default="headline",
                    help="general: DEHW's general-mesh features on the same chain (the contact band refined once "
                         "more -> hanging level, rotated support nodes, explicit transfer lists) with the same "
                         "coarse space (MULTISCALE_1 on the general tree)")
    ap.add_argument("--uneven", action="store_true",
                    help="group g (1 + g mod 3) times --nx cells long: subdomains of three sizes, packed onto the "
                         "ranks by LPT (partition.owner_for) as DEHW's uneven subdomains (not the headline)")
    ap.add_argument("--no-general", action="store_true",
                    help="skip the general-mesh line the N = 1 headline run adds (a child process, before the headline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream-ceiling", action="store_true", help="skip the same-process STREAM ceiling")
    ap.add_argument("--traffic-json", default=os.environ.get("DDPCA_TRAFFIC_JSON", str(ROOT / "profiles" / "traffic.json")),
                    help="PMC-derived HBM bytes per launch of the roofline kernel (profiles/make_traffic.py)")
    return ap.parse_args()


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one process per GPU)")
    import torch
    import torch.distributed as dist

    # the general-mesh line: its own process, before the headline allocates anything
    # on the host (each setup peaks at tens of GB), its JSON object attached to this line
    general_line = None
    if a.mesh == "headline" and world == 1 and not a.no_general:
        general_line = run_general_child(a)
    torch.cuda.set_device(local)  # the timing syncs below must hit this rank's GPU, not device 0
    if world > 1:
        # one node: RCCL's bootstrap over loopback (its data path is xGMI peer-to-peer either way);
        # an interface chosen by the launcher's environment wins
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        # host-side coordination only (barriers, the RCCL unique id, max-over-ranks timing); the
        # data path's exchanges are RCCL calls inside libddpca_amd on the solve stream
        dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module("ddpca-admm_amd")
    from importlib import import_module
    part = import_module("ddpca-admm_amd.partition")

    t_setup = time.perf_counter()
    general = a.mesh == "general"
    feat = dict(D.GENERAL_FEATURES) if general else {}
    P = D.headline_problem(groups=a.groups, nx=a.nx, ny=a.ny, nz=a.nz, gl=a.gl, fric=a.fric,
                           ip_contact=a.ip_contact, ip_glued=a.ip_glued, uneven=int(a.uneven), **feat)
    nip = sum(len(P.array("ip_w", ts)) for ts in range(P.nint))
    nsub = P.nsub
    # contiguous blocks for equal subdomains (worm/wheel pairs stay together), LPT by node count
    # when the sizes differ (--uneven; DEHW's 52 subdomains)
    owner = part.owner_for([len(P.array("coords", tv)) // 3 for tv in range(nsub)], world)
    # the option set of the rank with the most subdomains (all ranks run the same set)
    Hs = D.headline_options(max(list(owner).count(r) for r in range(world)))
    if a.smoother is None:
        a.smoother = Hs["smoother"]
    if a.nu is None:
        a.nu = Hs["nu"]
    if a.musc:
        P.set_coarse(a.musc, [a.dole] * nsub)
    P.ESTABLISH(owner, rank)
    mc = D.MCONTACT(P, device=local, rank=rank, nranks=world, owner=owner, smoother=a.smoother, nu=a.nu,
                    omega=-a.omega_scale, coarse_level=a.coarse_level,
                    iters_per_graph=a.iters_per_graph, warm_start=a.warm_start, precond_fp32=a.precond_fp32,
                    table_mode=a.table_mode)
    if world > 1:
        obj = [mc.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        mc.comm_init(obj[0])
    t_setup = time.perf_counter() - t_setup
    log(rank, f"setup {t_setup:.1f} s ({nip} integration points)")

    def barrier():
        if world > 1:
            dist.barrier()

    if a.warmup > 0:
        mc.CONTACT_ANALYSIS(a.warmup, check=False)
    log(rank, "warmup done")
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = mc.CONTACT_ANALYSIS(a.steps, check=False)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    log(rank, f"{n} ADMM iterations in {elapsed:.3f} s")
    tm = mc.timing()
    by = mc.bytes()  # algorithmic bytes of the timed iterations per phase (mcontact_gpu_bytes)
    phases = list(mc.BYTE_PHASES)
    if world > 1:
        t = torch.tensor([by[k] for k in phases], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        by.update({k: float(v) for k, v in zip(phases, t)})
    if world > 1:
        t = torch.tensor([elapsed, tm["dof_iterations"], tm["pcg_iterations"]], dtype=torch.float64)
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        dof_its, pcg_its = float(tsum[1]), float(tsum[2])
    else:
        dof_its, pcg_its = tm["dof_iterations"], tm["pcg_iterations"]
    dofs = [int(P.array("freeCount", tv)[-1]) if owner[tv] == rank else 0 for tv in range(nsub)]
    total_dofs = sum(dofs)
    if world > 1:
        t = torch.tensor([float(total_dofs)], dtype=torch.float64)
        dist.all_reduce(t)
        total_dofs = int(t[0])

    result = None
    if rank == 0:
        kern_ms = tm["spmv_kernel_ms"] / max(tm["spmv_samples"], 1.0)
        kbytes = tm["spmv_bytes_per_launch"]
        achieved = kbytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None
        # PMC-measured HBM bytes per launch of the same kernel on the same configuration
        # (profiles/make_traffic.py); ignored when it was measured on another configuration
        traffic, traffic_src = None, None
        if a.traffic_json and Path(a.traffic_json).exists():
            tj = json.loads(Path(a.traffic_json).read_text())
            if tj.get("config") == traffic_key(a):
                traffic = tj.get("hbm_bytes_per_launch")
                # PMC counters cannot be read inside this process (rocprofv3 --pmc is its own run):
                # the figure is the committed measurement of this kernel on this configuration
                traffic_src = f"replayed: {Path(a.traffic_json).relative_to(ROOT) if Path(a.traffic_json).is_relative_to(ROOT) else a.traffic_json}" \
                              f" ({tj.get('source', 'rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE')})"
        # this box's own STREAM ceiling, measured in this process after the timed region (SURVEY §8
        # d3): boxes of this pool stream at different rates, so frac_of_stream is the figure that
        # carries from one box to another; frac stays against the 8 TB/s spec peak
        ceiling = None
        if not a.no_stream_ceiling:
            ceiling = D.stream_ceiling(local)
            log(rank, f"STREAM ceiling: copy {ceiling['copy_gbs']:.0f} GB/s, read {ceiling['read_gbs']:.0f} GB/s")
        result = {
            "metric": "ADMM iters/sec",
            "value": n / elapsed,
            "unit": "ADMM it/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / n * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"dehw-synthetic{' general-mesh' if general else ''}{' uneven' if a.uneven else ''}: {nsub} subdomains x "
                             f"{total_dofs // nsub} DOF = {total_dofs} DOF, "
                             f"{a.groups} frictional contacts (mu={a.fric}) + {2 * (a.groups - 1)} glued interfaces, "
                             f"{nip} integration points ({nip / total_dofs:.2f} per DOF), "
                             f"{a.gl + 1 + (1 if general else 0)} MG levels, MGPIS-PCG rtol 1e-14"
                             + (", contact band refined once more (hanging level past the MGPIS hierarchy), "
                                "rotated support nodes, explicit transfer lists (DDPCA_LATTICE=0)" if general else "")),
                "subdomains": nsub,
                "dof": total_dofs,
                "interfaces": P.nint,
                "integration_points": nip,
                "ip_per_dof": nip / total_dofs,
                "mg_levels": a.gl + 1 + (1 if general else 0),
                "smoother": {0: "jacobi", 1: "block-jacobi", 2: "chebyshev"}[a.smoother] + f"({a.nu})" if a.smoother < 3
                else f"fine: multicolour block Gauss-Seidel (1 forward, 1 backward); below: block-jacobi({a.nu})"
                if a.smoother == 3 else
                f"fine: multicolour block SSOR (forward + backward before and after); below: block-jacobi({a.nu})",
                "pcg_x0": "previous solution" if a.warm_start else "zero",
                "vcycle_operator_storage": {0: "fp64", 1: "fp32",
                                            2: f"fp32, the {os.environ.get('DDPCA_H16_LEVELS', '3')} finest levels "
                                               "block-exponent fp16",
                                            3: f"fp32, the {os.environ.get('DDPCA_H16_LEVELS', '3')} finest levels "
                                               "block-scaled int8",
                                            4: f"fp32, the {os.environ.get('DDPCA_H16_LEVELS', '3')} finest levels "
                                               "block-scaled int8; the sweeps (" + ("" if general else "fine colour "
                                               "sweeps, ") + "block-Jacobi levels) gather fp32 copies of the iterate"}[a.precond_fp32],
                "operator_rows": "deduplicated table" if a.table_mode else "streamed",
                "coarse_space": f"interface-eliminated (muscSett={a.musc}, doleMcsc={a.dole})" if a.musc else "none",
                **({"hanging_dofs": int(sum(P.grid(tv).hangRows().shape[0] for tv in range(nsub) if owner[tv] == rank)),
                    "lattice_transfers": os.environ.get("DDPCA_LATTICE", "1") != "0"} if general else {}),
                "parallelism": f"dd{world}",
            },
            "mgpis_dof_iter_per_s": dof_its / elapsed,
            "pcg_iters_per_solve": pcg_its / max(n * nsub, 1),
            # this rank's subdomains in the last timed ADMM iteration (the state cpu_baseline prices)
            "pcg_iters_last_iteration": [int(v) for v in mc.get("pcg_iters")],
            "setup_s": t_setup,
            "mass_cg_iters_per_admm_iter": int(mc.get("mass_iters")[0]) / max(n, 1),
            # device time per ADMM iteration of the interface step (gamma, projection, aux / lambda
            # mass solves, MONITOR norms) and of the body balance (host wall, PCG + coarse space)
            "iface_ms_per_iter": tm["iface_ms"] / max(n, 1),
            "solve_ms_per_iter": tm["solve_ms"] / max(n, 1),
            "roofline": {
                "bound": "hbm",
                "kernel": "k_sell<kPcg> fine level (SELL-BSR3 SpMV q=Kz+beta q, p=z+beta p, p.q)",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": kbytes,
                "avg_launch_ms": kern_ms,
                "samples": int(tm["spmv_samples"]),
            },
        }
        if ceiling is not None:
            best = max(ceiling["copy_gbs"], ceiling["read_gbs"])
            result["roofline"].update({
                "stream_ceiling_gbs": {"copy": ceiling["copy_gbs"], "read": ceiling["read_gbs"],
                                       "bytes_per_buffer": ceiling["bytes_per_buffer"]},
                # against the higher of the two (the kernel's bytes are ~94 % reads)
                "frac_of_stream": achieved / best if achieved else None,
            })
        # whole-step roofline: the algorithmic bytes of EVERY kernel
        # of an ADMM iteration (byte model per kernel, DESIGN.md §3, summed over the members'
        # actual iteration counts) / the measured time per ADMM iteration / the HBM peak
        step_bytes = sum(by[k] for k in phases) / max(n, 1)
        step_s = elapsed / max(n, 1)
        split = {"fine_level_pcg": by["pcg_fine"], "coarse_levels_and_scalars": by["pcg_coarse"],
                 "coarse_space": by["coarse_space"], "mass_cg": by["mass_cg"],
                 "interface_rhs_monitor": by["interface"] + by["body_rhs"] + by["monitor"]}
        result["roofline"].update({
            "step_bytes": step_bytes,
            "step_achieved": step_bytes / step_s / 1e9,
            "step_frac": step_bytes / step_s / 1e9 / HBM_PEAK_GBS,
            "step_split_bytes": {k: v / max(n, 1) for k, v in split.items()},
            "pcg_launches_per_admm_iter": by["pcg_launches"] / max(n, 1),
        })
        if ceiling is not None:
            result["roofline"]["step_frac_of_stream"] = step_bytes / step_s / 1e9 / max(ceiling["copy_gbs"], ceiling["read_gbs"])
        if world == 1 and not a.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(P, mc)
        if general_line is not None:
            result["general_mesh"] = general_line
    # release device state before the process group
    del mc
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if result is not None:
        print(json.dumps(result), flush=True)


def run_general_child(a) -> dict:
    """The general-mesh line: bench.py --mesh general in a child process (DDPCA_LATTICE=0), same
    workload size, steps and warmup; its JSON object, or the failure."""
    import subprocess
    cmd = [sys.executable, str(Path(__file__).resolve()), "--mesh", "general", "--no-general", "--no-cpu-baseline",
           "--no-stream-ceiling", "--steps", str(a.steps), "--warmup", str(a.warmup), "--groups", str(a.groups),
           "--nx", str(a.nx), "--ny", str(a.ny), "--nz", str(a.nz), "--gl", str(a.gl), "--fric", str(a.fric),
           "--ip-contact", str(a.ip_contact), "--ip-glued", str(a.ip_glued),
           # precond_fp32 = 4: the colour sweeps' fp32 copy needs lattice fine transfers without band
           # mode, which the general line has not; its block-Jacobi levels take theirs (+5.5 % against
           # option 3, alternating in one call, profiles/r06q)
           "--precond-fp32", str(a.precond_fp32),
           "--traffic-json", str(ROOT / "profiles" / "traffic_general.json")]
    env = dict(os.environ, DDPCA_LATTICE="0")
    t0 = time.perf_counter()
    log(0, "general-mesh line (child process) ...")
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc={r.returncode}", "stderr_tail": r.stderr[-1500:]}
    j = json.loads(lines[-1])
    log(0, f"general-mesh line: {j.get('value', 0):.3f} ADMM it/s ({time.perf_counter() - t0:.0f} s incl. setup)")
    for k in ("n_gpus", "steps", "warmup", "higher_is_better", "scaling", "vs_baseline", "data"):
        j.pop(k, None)
    return j


def log(rank: int, msg: str) -> None:
    """Progress on stderr (stdout carries the one JSON line)."""
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def traffic_key(a) -> dict:
    # the roofline launch does not depend on musc / omega / coarse level; it does on the value layout
    k = dict(groups=a.groups, nx=a.nx, ny=a.ny, nz=a.nz, gl=a.gl, smoother=a.smoother, nu=a.nu,
             precond_fp32=a.precond_fp32, table_mode=a.table_mode, value_layout=VALUE_LAYOUT)
    if a.mesh != "headline":
        k["mesh"] = a.mesh
    return k


def cpu_baseline(P, mc, budget_s=20.0):
    """SGS-faithful CPU port (oracle/cpu_admm.py, MGPIS.h + MCONTACT.h) pricing one full ADMM
    iteration at the state the device run reached: sampled subdomain CG_SOLV(1) solves, the whole
    coarse-space correction and interface step.  `reference_equivalent` rescales it by the
    measured ratio of the reference's own CG_SOLV (oracle/_ref/ref_harness_portable, compiled from
    /root/reference's headers) to the port on the same BEAM mesh (profiles/cpu_calibration.py),
    timed ON THE GPU HOST at its 16 threads (profiles/r03_cpu_calibration_host.json); the
    container's 8-thread ratio is the fallback.  `reference_measured` is the reference's own
    CG_SOLV(1) (MGPIS.h:163-225) timed on this host on a wheel's and a worm's operators at the same
    state (oracle/_ref/ref_harness_portable time_cg_ops), the rest of the iteration by the port."""
    from oracle import cpu_admm
    exe = ROOT / "oracle" / "_ref" / "ref_harness_portable"
    try:
        res = cpu_admm.price_iteration(P, mc, budget_s, ref_exe=exe if exe.exists() else None)
    except (RuntimeError, OSError, ValueError, subprocess.TimeoutExpired) as e:  # the reference leg only
        print(f"[cpu_baseline] reference CG_SOLV leg failed: {e}", file=sys.stderr, flush=True)
        res = cpu_admm.price_iteration(P, mc, budget_s)
        res["reference_measured"] = {"error": str(e)[-300:]}
    res["host"] = host_cpu()
    # the reference's WHOLE ADMM iteration on this workload -- its unmodified CONTACT_ANALYSIS
    # (every subdomain's CG_SOLV(1) in its omp parallel for, the coarse correction, the interface
    # step, MONITOR, its text output) on the bench's operators at the device run's late state,
    # measured on a GPU box's host by profiles/ref_admm_time.py (minutes of CPU work: not rerun
    # here), replayed when it was measured on this workload
    full = ROOT / "profiles" / "ref_admm_full.json"
    if full.exists():
        j = json.loads(full.read_text())
        if j.get("dof") == P_dofs(P) and j.get("integration_points") == P_nip(P):
            its = j["iteration_s"]
            res["reference_full_iteration"] = {
                "value": j["value"], "unit": "ADMM it/s", "kind": "reference", "cores": j["threads"],
                "iteration_s": its, "cpu": j.get("cpu"), "host_cores": j.get("host_cores"),
                "source": f"replayed: {full.relative_to(ROOT)} (profiles/ref_admm_time.py, oracle/ref_admm_time.cpp: "
                          "the reference's own MCONTACT::CONTACT_ANALYSIS, text output included)",
                "sample": f"{len(its)} reference ADMM iterations from the device run's state after "
                          f"{j.get('device_iterations')} iterations: {[round(x, 1) for x in its]} s"}
    cal = ROOT / "profiles" / "r03_cpu_calibration_host.json"
    if not cal.exists():
        cal = ROOT / "profiles" / "r02_cpu_calibration.json"
    if cal.exists():
        c = json.loads(cal.read_text())
        res["calibration"] = {"ref_over_port": c["ref_over_port"], "mesh": c["mesh"], "threads": c["threads"],
                              "cpu": c.get("cpu"), "reference_s": c["reference"]["median_s"],
                              "port_s": c["port"]["median_s"], "source": str(cal.relative_to(ROOT))}
        res["reference_equivalent"] = res["value"] / c["ref_over_port"]
    return res


def P_dofs(P) -> int:
    return int(sum(int(P.array("freeCount", tv)[-1]) for tv in range(P.nsub)))


def P_nip(P) -> int:
    return int(sum(len(P.array("ip_w", ts)) for ts in range(P.nint)))


def host_cpu() -> dict:
    """The CPU the baseline ran on: model, the machine's physical cores (per socket x sockets) and
    the threads this process may use (the lease's OMP_NUM_THREADS on the GPU box)"""
    import re
    info = {"threads_used": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), "logical_cpus": os.cpu_count()}
    try:
        txt = open("/proc/cpuinfo").read()
        m = re.search(r"model name\s*:\s*(.+)", txt)
        cores = {int(c) for c in re.findall(r"cpu cores\s*:\s*(\d+)", txt)}
        sockets = {int(p) for p in re.findall(r"physical id\s*:\s*(\d+)", txt)}
        info.update({"model": m.group(1).strip() if m else None,
                     "physical_cores": (max(cores) * max(len(sockets), 1)) if cores else None,
                     "sockets": len(sockets) or None})
    except OSError:
        pass
    return info


if __name__ == "__main__":
    main()
