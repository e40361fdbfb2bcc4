"""Tune sweep throughput (BASELINE "Tune sweep" row): the reference's
``tune_mnist`` example (examples/ray_ddp_tune.py -- search space
layer_1 x layer_2 x lr x batch_size, TuneReportCheckpointCallback at every
validation end) run end to end on the local runtime, timed on the driver.

Reports trials/hour for the whole sweep, the per-trial wall time and how many
trials ran concurrently (trials x workers packed onto the visible GPUs).

    python scripts/bench_tune.py [--trials 4] [--workers 1] [--epochs 2] [--use-gpu 1]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))

from ray_lightning_accelerators_amd import runtime as ray  # noqa: E402

import ray_ddp_tune  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--warm", type=float, default=0.0, help="seconds to let the runtime pre-start its worker pool")
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--use-gpu", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=None, help="GPUs the runtime may pack trials onto")
    ap.add_argument("--share-gpu", type=int, default=0,
                    help="rehearsal: a virtual N-GPU ledger whose devices all map to GPU 0 (config 4's 4 trials x "
                         "2 workers on a 1-GPU box; gloo process groups, xGMI protocol over same-device IPC)")
    ap.add_argument("--diag", action="store_true",
                    help="worker reuse audit: every fit writes its process / communicator record "
                         "(RLA_WORKER_DIAG_DIR); checked per trial and summarised in the JSON")
    ap.add_argument("--diag-dir", default=None,
                    help="where --diag records go (default: a temp dir); workers also dump their "
                         "stacks there when a fit runs > 60 s (RLA_HANG_DUMP_DIR)")
    args = ap.parse_args()
    diag_dir = None
    if args.diag or args.diag_dir:
        args.diag = True
        diag_dir = args.diag_dir or tempfile.mkdtemp(prefix="rla_diag_")
        os.makedirs(diag_dir, exist_ok=True)
        diag_dir = os.path.abspath(diag_dir)
        os.environ["RLA_WORKER_DIAG_DIR"] = diag_dir
        os.environ.setdefault("RLA_HANG_DUMP_DIR", diag_dir)
    gpu = bool(args.use_gpu)
    if gpu:
        import torch

        n_gpus = args.gpus if args.gpus is not None else torch.cuda.device_count()
    else:
        n_gpus = 0
    os.environ.setdefault("TUNE_RESULTS_DIR", tempfile.mkdtemp())
    ncpu = max(16, (args.workers + 1) * args.trials)  # the box's 16-CPU share
    if gpu and args.share_gpu:
        n_gpus = args.share_gpu
        os.environ["RLA_PG_BACKEND"] = "gloo"  # RCCL refuses two ranks on one device
        ray.init(num_cpus=ncpu, _nodes=[{"ip": "127.0.0.1", "num_cpus": ncpu, "num_gpus": n_gpus,
                                         "gpu_ids": ["0"] * n_gpus, "resources": {}}])
    else:
        ray.init(num_cpus=ncpu, num_gpus=n_gpus)
    time.sleep(args.warm)  # a long-lived cluster has its worker pool warm; 0 = cold start counted
    t0 = time.perf_counter()
    _progress(t0, diag_dir)
    try:
        analysis = ray_ddp_tune.tune_mnist(os.path.join(tempfile.gettempdir(), "mnist_data_"), args.trials,
                                           args.epochs, args.workers, gpu)
        wall = time.perf_counter() - t0  # the sweep: first trial launched .. last result in
    finally:
        t1 = time.perf_counter()
        ray.shutdown()
        shutdown_s = time.perf_counter() - t1
    df = analysis.results_df
    iters = [int(v) for v in df["training_iteration"]] if "training_iteration" in df else []
    audit = None
    if diag_dir:
        audit = _audit(diag_dir, analysis, args)
    print(json.dumps({
        "metric": "Tune sweep trials/hour (tune_mnist, RayAccelerator workers)",
        "value": round(args.trials / wall * 3600.0, 1), "unit": "trials/hour", "trials": args.trials,
        "workers_per_trial": args.workers, "gpus": n_gpus, "epochs_per_trial": args.epochs,
        "wall_s": round(wall, 2), "runtime_shutdown_s": round(shutdown_s, 2), "pool_warm_s": args.warm, "virtual_gpus_on_one": args.share_gpu, "s_per_trial": round(wall / args.trials, 2), "reports_per_trial": iters,
        "best_config": analysis.best_config, "data": "synthetic", "reuse_audit": audit}), flush=True)
    if audit is not None and not audit["ok"]:
        raise SystemExit(f"worker reuse audit failed: {audit['problems']}")


def _progress(t0, diag_dir, every_s: float = 15.0):
    """A progress line on stderr every ``every_s`` (elapsed, fits finished so far):
    a long sweep keeps telling the caller it is alive, and a stall shows where."""
    import glob
    import threading

    def run():
        while True:
            time.sleep(every_s)
            fits = len(glob.glob(os.path.join(diag_dir, "*.json"))) if diag_dir else None
            print(f"[bench_tune] {time.perf_counter() - t0:.0f} s, fits recorded: {fits}", file=sys.stderr,
                  flush=True)

    threading.Thread(target=run, daemon=True).start()


def _audit(diag_dir, analysis, args):
    """Per trial: max_epochs reports and a checkpoint; per fit: every rank on a fresh
    communicator (a new object, no error, rank / world as the trial's), the exchange
    region re-armed; plus how many fits recycled processes served."""
    import glob

    recs = [json.load(open(p)) for p in sorted(glob.glob(os.path.join(diag_dir, "*.json")))]
    problems = []
    for t in analysis.trials:
        if len(t.results) != args.epochs:
            problems.append(f"{t.trial_id}: {len(t.results)} reports, expected {args.epochs}")
        if not t.checkpoint or not os.path.exists(t.checkpoint):
            problems.append(f"{t.trial_id}: no checkpoint")
    comm_ids = {}
    for r in recs:
        if r["world"] != args.workers:
            problems.append(f"fit {r}: world {r['world']}")
        if args.workers > 1 and args.use_gpu:
            if r["comm_id"] is None or r["comm_error_state"] != 0:
                problems.append(f"pid {r['pid']} fit {r['fit_in_process']}: communicator {r['comm']}")
            if r["fused_dp"] and r["dp_region_rearms"] < 1:
                problems.append(f"pid {r['pid']} fit {r['fit_in_process']}: exchange region never re-armed")
            key = (r["pid"], r["comm_id"])
            if key in comm_ids:
                problems.append(f"pid {r['pid']}: communicator reused across fits {comm_ids[key]} and "
                                f"{r['fit_in_process']}")
            comm_ids[key] = r["fit_in_process"]
    recycled = sum(1 for r in recs if r["fit_in_process"] > 1)
    return {"ok": not problems, "problems": problems[:10], "fits": len(recs), "processes": len({r["pid"] for r in recs}),
            "fits_on_recycled_workers": recycled, "max_fits_per_process": max((r["fit_in_process"] for r in recs),
                                                                            default=0),
            "fused_dp_fits": sum(1 for r in recs if r["fused_dp"]),
            "ckpt_writer_takeovers": max((r.get("ckpt_writer_takeovers", 0) for r in recs), default=0),
            "dp_protos": sorted({r["dp_proto"] for r in recs if r["dp_proto"]})}


if __name__ == "__main__":
    main()
