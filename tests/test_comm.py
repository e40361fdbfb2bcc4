"""Native comm engine (csrc/comm/*): xGMI one-shot allreduce, fusion engine,
RCCL communicator, and the Python routing layer (parallel/comm.py).

The GPU tests run TWO ranks on the box's single MI355X: both processes map each
other's uncached receive regions through hipIpcOpenMemHandle exactly as peer
GPUs do over xGMI (same protocol, same kernels; only the physical link
differs).  RCCL itself refuses two ranks on one device, so its path is tested
at world size 1 plus the routing fallback.
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

gpu = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group(backend, rank=rank, world_size=world)


# ---------------------------------------------------------------- CPU (gloo)
def _cpu_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from ray_lightning_accelerators_amd.parallel.comm import make_allreduce

        f = make_allreduce(average=True)
        t = torch.full((10,), float(rank + 1))
        f(t)
        q.put((rank, t.tolist()))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_make_allreduce_falls_back_to_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_cpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert out[0] == [1.5] * 10 and out[1] == [1.5] * 10, out


# ---------------------------------------------------------------- GPU (IPC)
def _gpu_worker(rank, world, port, q, mode):
    try:
        torch.cuda.set_device(0)
        _init(rank, world, port)
        from ray_lightning_accelerators_amd.parallel.comm import NativeCommunicator

        ts_modes = ("twoshot", "twoshot_timeout", "reducer_ts", "reducer_bf16", "validation_fault")
        if mode == "validation_fault":
            # rank 1 skips its validation launches: rank 0's bounded polls time out (error
            # word latched); both paths must be dropped on BOTH ranks and the error cleared
            os.environ["RLA_FAULT_XGMI_VALIDATION"] = "1"
        if mode == "matrix":
            comm = NativeCommunicator(use_rccl=False, use_xgmi=True, xgmi_bytes=2 << 20, twoshot_bytes=32 << 20,
                                      spin_limit=1 << 22)
        else:
            comm = NativeCommunicator(use_rccl=False, use_xgmi=True,
                                      xgmi_bytes=(1 << 10) if mode in ts_modes else (1 << 20),
                                      twoshot_bytes=(4 << 20) if mode in ts_modes else 0,
                                      # short bounded polls only where a dead peer is simulated: elsewhere a
                                      # slow-starting peer process must not trip the timeout (a timed-out
                                      # block skips its reduction -- comm.check() reports it)
                                      spin_limit=(1 << 20) if ("timeout" in mode or mode == "validation_fault") else (1 << 24))
        res = {"xgmi": comm.xgmi, "twoshot": comm.twoshot}
        dev = torch.device("cuda", 0)
        if mode == "twoshot":
            # exact fp32 sums of integer-valued data, ragged sizes (chunk tails, empty chunks)
            for n in (1, 3, 4, 5, 17, 255, 4099, 70001, 262147, 1000003):
                base = torch.arange(n, device=dev, dtype=torch.float32) % 97
                x = base * (rank + 1) + rank
                comm._c.allreduce_twoshot(x, False)
                torch.cuda.synchronize()
                want = base * (world * (world + 1) / 2) + sum(range(world))
                res[f"fp32_{n}"] = bool(torch.equal(x, want))
            # router: small buckets one-shot, larger ones two-shot, all exact
            routes = {}
            for n in (200, 5000, 300001):
                x = torch.full((n,), float(rank + 1), device=dev)
                routes[n] = comm.route(x)
                comm.allreduce_(x)
                torch.cuda.synchronize()
                res[f"routed_{n}"] = bool(torch.all(x == world * (world + 1) / 2))
            res["routes"] = routes
            # bf16 wire: fp32 accumulate of bf16-rounded inputs, identical bits on every rank
            g = torch.Generator(device=dev).manual_seed(10 + rank)
            x = torch.randn(123457, device=dev, generator=g)
            ref = [torch.randn(123457, device=dev, generator=torch.Generator(device=dev).manual_seed(10 + r))
                   .to(torch.bfloat16).float() for r in range(world)]
            want = sum(ref[1:], ref[0]).to(torch.bfloat16).float()
            comm.allreduce_(x, bf16_wire=True)
            torch.cuda.synchronize()
            res["bf16_close"] = bool(torch.allclose(x, want, rtol=1e-2, atol=1e-2))
            res["bf16_bytes"] = x.cpu().numpy().tobytes()
            # hipGraph capture: replays advance the per-block generations
            y = torch.ones(300001, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                comm.allreduce_(y)
            for k in range(3):
                y.fill_(rank + 1.0 + k)
                gr.replay()
                torch.cuda.synchronize()
                res[f"graph{k}"] = bool(torch.all(y == world * (world + 1) / 2 + world * k).item())
            comm.check()
        elif mode == "matrix":
            # correctness matrix: 4 B ... 32 MiB x {one-shot, two-shot fp32,
            # two-shot bf16 wire, router}; integer-valued data so fp32 sums are exact
            bad = []
            # 32 Mi floats = 128 MiB: above the two-shot region -> region-sized launches
            sizes = [1, 2, 7, 64, 1000, 4096 + 3, 65536, 262147, 1 << 20, (1 << 21) + 5, 8 << 20,
                     (20 << 20) + 12, 32 << 20]
            if world >= 8:  # eight ranks time-slice one device: one region-sized size is enough
                sizes = sizes[:-1]
            for n in sizes:
                base = (torch.arange(n, device=dev, dtype=torch.float32) % 31) - 15
                want = base * (world * (world + 1) / 2)
                if world == 1:
                    # world 1: every path is the identity (no peers, no region)
                    res.setdefault("big_routes", []).append(comm.route(base))
                    paths = ["router", "bf16_routed"]
                elif n > comm.twoshot_capacity:
                    res.setdefault("big_routes", []).append(comm.route(base))
                    paths = ["router", "bf16_routed"]
                else:
                    paths = ["router", "twoshot", "bf16"] + (["oneshot"] if n <= comm.xgmi_capacity else [])
                for path in paths:
                    x = base * (rank + 1)
                    if path == "oneshot":
                        comm._c.allreduce_xgmi(x)
                    elif path == "twoshot":
                        comm._c.allreduce_twoshot(x, False)
                    elif path == "bf16":
                        comm._c.allreduce_twoshot(x, True)  # |values| <= 150: exact in bf16
                    elif path == "bf16_routed":
                        comm.allreduce_(x, bf16_wire=True)
                    else:
                        comm.allreduce_(x)
                    torch.cuda.synchronize()
                    if not torch.equal(x, want):
                        bad.append((n, path, float((x - want).abs().max())))
            res["bad"] = bad
            comm.check()
        elif mode == "validation_fault":
            res["fallbacks"] = list(comm.fallbacks)
            res["state_after_setup"] = comm._c.error_state()
            x = torch.full((70001,), float(rank + 1), device=dev)
            res["route"] = comm.route(x)
            comm.allreduce_(x)  # gloo bootstrap fallback (RCCL refuses 2 ranks on one device)
            torch.cuda.synchronize()
            res["sum_ok"] = bool(torch.all(x == world * (world + 1) / 2))
            comm.check()  # must not raise: the latched timeout was cleared
            res["checked"] = True
        elif mode == "twoshot_timeout":
            x = torch.ones(100000, device=dev)
            if rank == 0:
                comm._c.allreduce_twoshot(x, False)  # the peers never join: bounded polls give up
                torch.cuda.synchronize()
            dist.barrier()
            res["state"] = comm._c.error_state()
        elif mode in ("reducer_ts", "reducer_bf16"):
            # GradSynchronizer buckets above the (tiny) one-shot area -> C++ reducer -> two-shot
            from ray_lightning_accelerators_amd.parallel import comm as comm_mod
            from ray_lightning_accelerators_amd.parallel.arena import ParamArena
            from ray_lightning_accelerators_amd.parallel.ddp import GradSynchronizer

            comm_mod._default = comm

            def make():
                torch.manual_seed(0)
                return torch.nn.Sequential(torch.nn.Linear(256, 300), torch.nn.ReLU(), torch.nn.Linear(300, 77),
                                           torch.nn.ReLU(), torch.nn.Linear(77, 5)).to(dev)

            def data(r):
                g = torch.Generator().manual_seed(300 + r)
                return torch.randn(32, 256, generator=g).to(dev), torch.randn(32, 5, generator=g).to(dev)

            model = make()
            arena = ParamArena(model)
            gdt = "bf16" if mode == "reducer_bf16" else "fp32"
            sync = GradSynchronizer(model, arena, bucket_cap_mb=0.05, grad_dtype=gdt, average_in_optimizer=False)
            res["native_reducer"] = sync._native is not None
            res["buckets"] = len(sync.buckets)
            res["bucket_routes"] = sorted({comm.route(arena.grad[b.start:b.end]) for b in sync.buckets})
            for _ in range(2):
                arena.zero_grad()
                sync.prepare_for_backward()
                x, y = data(rank)
                torch.nn.functional.mse_loss(model(x), y).backward()
                sync.finish()
            ref = make()
            for r in range(world):
                x, y = data(r)
                (torch.nn.functional.mse_loss(ref(x), y) / world).backward()
            torch.cuda.synchronize()
            tol = 2e-2 if gdt == "bf16" else 1e-6
            res["match"] = all(bool(torch.allclose(p.grad, q.grad, atol=tol, rtol=tol)) for p, q in
                               zip(model.parameters(), ref.parameters()))
            res["grad_bytes"] = arena.grad.cpu().numpy().tobytes()
            comm.check()
        elif mode == "allreduce":
            for n in (1, 3, 4, 1024, 27882, 27884, 262143):  # incl. the 32/64 MLP arena (27,882)
                x = torch.arange(n, device=dev, dtype=torch.float32) * 0.5 + rank
                comm.allreduce_(x)
                torch.cuda.synchronize()
                want = torch.arange(n, device=dev, dtype=torch.float32) * 0.5 * world + sum(range(world))
                res[n] = bool(torch.equal(x, want))
            # graph capture: replays advance the device-side generation counters
            y = torch.ones(27884, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                comm.allreduce_(y)
            for k in range(3):
                y.fill_(rank + 1.0)
                g.replay()
                torch.cuda.synchronize()
                res[f"graph{k}"] = bool(torch.all(y == world * (world + 1) / 2).item())
            comm.check()
        elif mode == "fusion":
            eng = comm.fusion_engine(fusion_bytes=64 << 10)
            ts = [torch.full((n,), float(rank + 1), device=dev) for n in (3, 5000, 17, 40000, 8, 1)]
            hs = [eng.submit(t, 1.0 / world) for t in ts]
            eng.flush()
            for h, t in zip(hs, ts):
                assert eng.wait(h, t)
            torch.cuda.synchronize()
            want = (world + 1) / 2
            res["fused"] = all(bool(torch.allclose(t, torch.full_like(t, want))) for t in ts)
            res["batches"] = eng.batches_executed
            res["fingerprint"] = eng.fingerprint
            eng.drain()
        elif mode == "hvd":
            # Horovod DistributedOptimizer on the C++ fusion engine vs. a local reference
            os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), HOROVOD_FUSION_THRESHOLD="4096")
            import ray_lightning_accelerators_amd.horovod as hvd
            from ray_lightning_accelerators_amd.parallel import comm as comm_mod

            comm_mod._default = comm  # the group is up; reuse this rank's communicator
            hvd.init()

            def make():
                torch.manual_seed(0)
                return torch.nn.Sequential(torch.nn.Linear(64, 33), torch.nn.ReLU(),
                                           torch.nn.Linear(33, 5)).to(dev)

            def data(r):
                g = torch.Generator().manual_seed(100 + r)
                return torch.randn(16, 64, generator=g).to(dev), torch.randn(16, 5, generator=g).to(dev)

            model = make()
            opt = hvd.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                                           named_parameters=model.named_parameters())
            # the engine comes up at the first bucket launch (lazily: a step without
            # autograd never creates its stream); the communicator is bound now
            res["native_engine"] = opt._hvd_state._engine_comm is not None
            for _ in range(3):
                x, y = data(rank)
                opt.zero_grad()
                torch.nn.functional.mse_loss(model(x), y).backward()
                opt.step()
            ref = make()
            ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
            for _ in range(3):
                ropt.zero_grad()
                for r in range(world):
                    x, y = data(r)
                    (torch.nn.functional.mse_loss(ref(x), y) / world).backward()
                ropt.step()
            torch.cuda.synchronize()
            res["maxdiff"] = max(float((a - b).abs().max()) for a, b in zip(model.parameters(), ref.parameters()))
            comm.check()
            res["match"] = all(bool(torch.allclose(a, b, atol=1e-5)) for a, b in
                               zip(model.parameters(), ref.parameters()))
            res["native_engine"] = res["native_engine"] and opt._hvd_state.engine is not None
            res["batches"] = opt._hvd_state.engine.batches_executed if res["native_engine"] else 0
        elif mode in ("reducer", "reducer_check"):
            # GradSynchronizer on the C++ reducer: several in-order buckets, averaged grads
            # (reducer_check: the Python path with the stream-ordering race detector on)
            from ray_lightning_accelerators_amd.config import RLAConfig, set_config
            from ray_lightning_accelerators_amd.parallel import comm as comm_mod

            if mode == "reducer_check":
                set_config(RLAConfig(check_streams=True))
            from ray_lightning_accelerators_amd.parallel.arena import ParamArena
            from ray_lightning_accelerators_amd.parallel.ddp import GradSynchronizer

            comm_mod._default = comm

            def make():
                torch.manual_seed(0)
                return torch.nn.Sequential(torch.nn.Linear(64, 130), torch.nn.ReLU(), torch.nn.Linear(130, 7),
                                           torch.nn.ReLU(), torch.nn.Linear(7, 3)).to(dev)

            def data(r):
                g = torch.Generator().manual_seed(200 + r)
                return torch.randn(16, 64, generator=g).to(dev), torch.randn(16, 3, generator=g).to(dev)

            model = make()
            arena = ParamArena(model)
            sync = GradSynchronizer(model, arena, bucket_cap_mb=100 / 2 ** 20, average_in_optimizer=False)
            res["native_reducer"] = sync._native is not None
            res["buckets"] = len(sync.buckets)
            for _ in range(2):
                arena.zero_grad()
                sync.prepare_for_backward()
                x, y = data(rank)
                torch.nn.functional.mse_loss(model(x), y).backward()
                # overlap: buckets are launched from the grad hooks DURING backward,
                # not by finish()
                res["launched_in_backward"] = (sync._native.launched if sync._native is not None
                                               else sum(b.work is not None for b in sync.buckets))
                sync.finish()
            ref = make()
            for r in range(world):
                x, y = data(r)
                (torch.nn.functional.mse_loss(ref(x), y) / world).backward()
            torch.cuda.synchronize()
            res["match"] = all(bool(torch.allclose(p.grad, q.grad, atol=1e-6)) for p, q in
                               zip(model.parameters(), ref.parameters()))
            res["launched"] = sync._native.launched if sync._native is not None else 0
            res["probes"] = sync.probes_checked
        elif mode in ("mlp_dp", "mlp_dp_timeout"):
            # fused data-parallel MLP step (gradient exchange inside the tail kernel)
            # vs. the split head / tail(grad) / allreduce / tail(adam) path
            from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine

            g = torch.Generator().manual_seed(7)
            xs = torch.randint(0, 256, (2048, 784), dtype=torch.uint8, generator=g)
            ys = torch.randint(0, 10, (2048,), generator=g)
            from ray_lightning_accelerators_amd.ops.fused_mlp import mlp3_dp_capacity

            ctx = comm.dp_context(mlp3_dp_capacity(32, 64))
            res["dp_ctx"] = ctx is not None

            bsz = int(os.environ.get("RLA_TEST_DP_BATCH", "64"))  # <= 32: the one-launch DP step

            def make(dp):
                e = FusedMLPEngine(32, 64, bsz, lr=1e-2, device=dev, world_size=world, rank=rank,
                                   allreduce=comm.allreduce_, dp_context=ctx if dp else None,
                                   dp_rearm=comm.dp_rearm if dp else None)
                e.set_data(xs, ys, shuffle=True)
                return e

            if mode == "mlp_dp_timeout":
                e = make(True)
                if rank == 0:  # rank 1 never runs the step: the in-kernel poll must give up
                    e.run(1)
                    torch.cuda.synchronize()
                dist.barrier()
                res["state"] = comm._c.error_state()
            else:
                e_dp, e_ref = make(True), make(False)
                res["dp_mode"] = e_dp.dp_ctx is not None
                res["one_launch_dp"] = e_dp.one_launch_dp
                res["proto"] = e_dp.dp_proto
                # granule / flags carry exact fp32; packed / owner round each wire value to
                # 4 ulp of fp32 (2^-22 relative), which Adam's normalised update passes on
                wire_tol = 1e-6 if e_dp.dp_proto in ("granule", "wave", "all") or not e_dp.one_launch_dp else 2e-5
                e_dp.run(6)
                e_ref.run(6)
                torch.cuda.synchronize()
                res["match"] = bool(torch.allclose(e_dp.params, e_ref.params, atol=wire_tol, rtol=0))
                res["maxdiff"] = float((e_dp.params - e_ref.params).abs().max())
                res["loss"] = e_dp.recent_stats(6)[:, 0].tolist()
                # graph replays continue the same trajectory
                ok = e_dp.capture()  # runs one real (warm-up) step
                e_ref.run(1)
                e_dp.run(4)
                e_ref.run(4)
                torch.cuda.synchronize()
                res["graph"] = ok
                res["match_graph"] = bool(torch.allclose(e_dp.params, e_ref.params, atol=10 * wire_tol, rtol=0))
                # owner: each element's Adam state lives on its owner until consolidated
                e_dp.sync_optimizer_state()
                torch.cuda.synchronize()
                res["m_match"] = bool(torch.allclose(e_dp.exp_avg, e_ref.exp_avg, atol=10 * wire_tol, rtol=1e-3))
                res["params"] = e_dp.params.cpu().numpy().tobytes()  # no shared-memory fds through the queue
                res["mv"] = torch.cat([e_dp.exp_avg, e_dp.exp_avg_sq]).cpu().numpy().tobytes()
                comm.check()
                e_dp.check()
        elif mode == "mlp_fidelity":
            # Step1DP at world 2 against fp32 autograd of BOTH ranks' batches (the DDP
            # average), every step over 2+ epochs
            import torch.nn.functional as F

            from ray_lightning_accelerators_amd.models.data import synthetic_mnist
            from ray_lightning_accelerators_amd.ops import fused_mlp
            from ray_lightning_accelerators_amd.parallel.mlp_engine import FusedMLPEngine, shard_indices

            L1, L2, B = 32, 64, 32
            x, y = synthetic_mnist(2 * B * 16 + 5, seed=14)
            ctx = comm.dp_context(fused_mlp.mlp3_dp_capacity(L1, L2))
            e = FusedMLPEngine(L1, L2, B, lr=1e-3, device=dev, world_size=world, rank=rank,
                               allreduce=comm.allreduce_, dp_context=ctx, dp_rearm=comm.dp_rearm,
                               dp_proto=os.environ.get("RLA_DP_PROTO", "packed"))
            e.set_data(x, y, shuffle=True)
            e.broadcast_from(0)
            res["one_launch_dp"] = e.one_launch_dp
            names = ("W1", "b1", "W2", "b2", "W3", "b3")

            def ref_grad(flat, idx):
                p = {k: v.clone().requires_grad_(True) for k, v in
                     zip(names, fused_mlp.mlp_unpack(flat.cpu(), L1, L2).values())}
                h = torch.relu(F.linear(x[idx].float() / 255.0, p["W1"], p["b1"]))
                h = torch.relu(F.linear(h, p["W2"], p["b2"]))
                F.nll_loss(torch.log_softmax(F.linear(h, p["W3"], p["b3"]), 1), y[idx]).backward()
                return torch.cat([p[k].grad.reshape(-1) for k in names])

            worst = {k: 0.0 for k in names}
            b1 = e.betas[0]
            nb = e.n_batches
            for _ in range(2 * nb + 3):
                epoch, cur = e.epoch, e.step_in_epoch
                p0, m0 = e.params.clone(), e.exp_avg.clone()
                e.step()
                g = (e.exp_avg - b1 * m0) / (1 - b1)
                ref = sum(ref_grad(p0, shard_indices(x.size(0), world, r, epoch, e.seed, True)[cur * B:(cur + 1) * B])
                          for r in range(world)) / world
                for k, a, b in zip(names, fused_mlp.mlp_unpack(g.cpu(), L1, L2).values(),
                                   fused_mlp.mlp_unpack(ref, L1, L2).values()):
                    e_k = (a - b).norm().item() / max(b.norm().item(), 1e-12)
                    # NaN-proof: max(0.0, nan) is 0.0, so a non-finite error is recorded as inf
                    worst[k] = max(worst[k], e_k) if math.isfinite(e_k) else math.inf
            torch.cuda.synchronize()
            comm.check()
            e.check()
            res["worst"] = worst
            res["params"] = e.params.cpu().numpy().tobytes()
        elif mode == "bcast_exact":
            # DDP buffer broadcast without RCCL (ranks share the device): int64 counters
            # above 2^24 and fp64 buffers arrive bit-exact, fp32 too
            from ray_lightning_accelerators_amd.parallel import comm as comm_mod
            from ray_lightning_accelerators_amd.parallel.arena import ParamArena
            from ray_lightning_accelerators_amd.parallel.ddp import GradSynchronizer

            comm_mod._default = comm
            m = torch.nn.Linear(8, 4).to(dev)
            m.register_buffer("big", torch.tensor([2 ** 40 + 12345 + rank, -7 - rank, 2 ** 24 + 1], device=dev))
            m.register_buffer("f64", torch.tensor([1.0 + 1e-12 * (rank + 1), -3.5e-300], dtype=torch.float64,
                                                  device=dev))
            m.register_buffer("f32", torch.full((5,), 0.1 * (rank + 1), device=dev))
            # 1-byte dtypes with an odd element count (no 16-bit view)
            m.register_buffer("u8", torch.tensor([255, rank, 7], dtype=torch.uint8, device=dev))
            m.register_buffer("flag", torch.tensor([rank == 0, rank != 0, True], device=dev))
            sync = GradSynchronizer(m, ParamArena(m), bucket_cap_mb=1.0)
            sync._broadcast_buffers()
            torch.cuda.synchronize()
            res["big"] = m.big.tolist() == [2 ** 40 + 12345, -7, 2 ** 24 + 1]
            res["f64"] = m.f64.tolist() == [1.0 + 1e-12, -3.5e-300]
            res["f32"] = bool(torch.all(m.f32 == torch.tensor(0.1, device=dev)))
            res["u8"] = m.u8.tolist() == [255, 0, 7]
            res["bool"] = m.flag.tolist() == [True, False, True]
            comm.check()
        elif mode == "timeout":
            x = torch.ones(1024, device=dev)
            if rank == 0:
                comm.allreduce_(x)  # rank 1 never joins: the bounded poll must give up
                torch.cuda.synchronize()
            dist.barrier()
            res["state"] = comm._c.error_state()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_gpu(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_gpu_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r, v = q.get(timeout=300)
        out[r] = v
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    for r, v in out.items():
        assert isinstance(v, dict), f"rank {r} failed:\n{v}"
    return out


@gpu
def test_xgmi_oneshot_allreduce_two_ranks():
    out = _run_gpu("allreduce")
    for r, res in out.items():
        assert res["xgmi"], res
        assert all(v for k, v in res.items() if k != "twoshot"), (r, res)


@gpu
def test_fusion_engine_two_ranks():
    out = _run_gpu("fusion")
    assert out[0]["fused"] and out[1]["fused"], out
    assert out[0]["fingerprint"] == out[1]["fingerprint"]
    assert out[0]["batches"] >= 2  # 64 KiB threshold splits the 6 requests


@gpu
def test_horovod_optimizer_on_native_fusion_engine():
    out = _run_gpu("hvd")
    for r, res in out.items():
        assert res["native_engine"] and res["match"], (r, res)
        assert res["batches"] >= 6  # 3 steps x >= 2 fusion buckets (4 KiB threshold)


@gpu
def test_ddp_native_reducer_two_ranks():
    out = _run_gpu("reducer")
    for r, res in out.items():
        assert res["native_reducer"] and res["match"], (r, res)
        assert res["buckets"] >= 3 and res["launched"] == 2 * res["buckets"]
        # every bucket went out from the hooks while backward was still running
        assert res["launched_in_backward"] == 2 * res["buckets"], res


@gpu
def test_ddp_stream_ordering_checker_two_ranks():
    out = _run_gpu("reducer_check")
    for r, res in out.items():
        assert not res["native_reducer"] and res["match"], (r, res)
        assert res["probes"] == 2 * res["buckets"], (r, res)


@gpu
def test_xgmi_dead_peer_times_out_instead_of_hanging():
    out = _run_gpu("timeout")
    assert out[0]["state"] == 1 and out[1]["state"] == 0, out


@gpu
@pytest.mark.parametrize("proto,batch", [("granule", 64), ("wave", 64), ("granule", 32), ("wave", 32),
                                         ("packed", 32), ("owner", 32)])
def test_fused_dp_mlp_step_matches_split_allreduce(proto, batch, monkeypatch):
    # granule: tagged 8-byte words, no fences; wave: flags + one fencing wave (two-launch);
    # packed: wave-positioned one-shot, two values per granule (default); owner:
    # reduce-scatter to the task's owner, Adam there, all-gather of the weights.
    # batch 32 + granule / packed / owner: the one-launch DP step (kind Step1DP)
    monkeypatch.setenv("RLA_DP_PROTO", proto)
    monkeypatch.setenv("RLA_TEST_DP_BATCH", str(batch))
    out = _run_gpu("mlp_dp")
    for r, res in out.items():
        assert res["dp_ctx"] and res["dp_mode"], (r, res)
        assert res["one_launch_dp"] == (batch <= 32 and proto in ("granule", "packed", "owner")), (r, res)
        info = {k: v for k, v in res.items() if k not in ("params", "mv")}
        assert res["match"] and res["match_graph"] and res["m_match"], (r, info)
        assert res["graph"]
    # replicas stay bitwise identical (every rank sums the tiles in rank order / the
    # owner's weights are everyone's), Adam state too once consolidated
    assert out[0]["params"] == out[1]["params"]
    assert out[0]["mv"] == out[1]["mv"]


@gpu
def test_fused_dp_one_launch_grads_vs_fp32_autograd_two_ranks(monkeypatch):
    """Step1DP (packed, 2 ranks) applies the DDP-averaged gradient of both ranks'
    batches: per tensor within the bf16 bounds of the one-rank kernel test."""
    from test_mlp3 import GRAD_BOUND, _fidelity_log

    monkeypatch.setenv("RLA_DP_PROTO", "packed")
    out = _run_gpu("mlp_fidelity")
    for r, res in out.items():
        assert res["one_launch_dp"], (r, res)
        for k, v in res["worst"].items():
            assert v < GRAD_BOUND[k], (r, k, res["worst"])
    _fidelity_log("dp_two_ranks_packed_grads", {"max_rel_err": out[0]["worst"]})
    assert out[0]["params"] == out[1]["params"]


@gpu
@pytest.mark.parametrize("batch,proto", [(64, "granule"), (32, "granule"), (32, "packed"), (32, "owner")])
def test_fused_dp_mlp_step_dead_peer_times_out(batch, proto, monkeypatch):
    monkeypatch.setenv("RLA_TEST_DP_BATCH", str(batch))
    monkeypatch.setenv("RLA_DP_PROTO", proto)
    out = _run_gpu("mlp_dp_timeout")
    assert out[0]["state"] == 1 and out[1]["state"] == 0, out


@gpu
@pytest.mark.parametrize("world", [2, 3])
def test_xgmi_twoshot_allreduce(world):
    out = _run_gpu("twoshot", world=world)
    for r, res in out.items():
        assert res["xgmi"] and res["twoshot"], (r, {k: v for k, v in res.items() if k != "bf16_bytes"})
        bad = {k: v for k, v in res.items() if v is False}
        assert not bad, (r, bad)
        assert res["routes"] == {200: "oneshot", 5000: "twoshot", 300001: "twoshot"}, res["routes"]
    # bf16 wire: every replica holds the same bits
    assert len({res["bf16_bytes"] for res in out.values()}) == 1


@gpu
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_comm_correctness_matrix(world):
    """worlds 1 / 2 / 4 / 8 x {one-shot, two-shot fp32, two-shot
    bf16 wire, router} x 4 B ... 128 MiB, every rank-class (NW) instance of the xGMI
    kernels; ranks share the one device (IPC of uncached regions, same code path)."""
    out = _run_gpu("matrix", world=world)
    assert len(out) == world
    for r, res in out.items():
        assert isinstance(res, dict), (r, res)
        if world == 1:
            assert set(res["big_routes"]) == {"none"} and not res["bad"], (r, res)
            continue
        assert res["xgmi"] and res["twoshot"], (r, res)
        assert not res["bad"], (r, res["bad"][:10])
        n_big = 1 if world >= 8 else 2
        assert res["big_routes"] == ["twoshot"] * n_big, (r, res["big_routes"])  # no RCCL: chunked two-shot


@gpu
def test_buffer_broadcast_without_rccl_is_exact():
    out = _run_gpu("bcast_exact")
    for r, res in out.items():
        assert isinstance(res, dict) and res["big"] and res["f64"] and res["f32"], (r, res)
        assert res["u8"] and res["bool"], (r, res)


@gpu
def test_failed_xgmi_validation_falls_back_cleanly():
    """a validation timeout latched the error word for good, so a run
    that correctly fell back still failed at the first ``check()``."""
    out = _run_gpu("validation_fault")
    for r, res in out.items():
        assert not res["xgmi"] and not res["twoshot"], (r, res)
        assert res["fallbacks"] == ["xGMI one-shot", "xGMI two-shot"], (r, res)
        assert res["state_after_setup"] == 0 and res["checked"], (r, res)
        assert res["route"] == "torch" and res["sum_ok"], (r, res)


@gpu
def test_xgmi_twoshot_dead_peer_times_out():
    out = _run_gpu("twoshot_timeout")
    assert out[0]["state"] == 1 and out[1]["state"] == 0, out


@gpu
@pytest.mark.parametrize("mode", ["reducer_ts", "reducer_bf16"])
def test_ddp_reducer_over_twoshot(mode):
    out = _run_gpu(mode)
    for r, res in out.items():
        assert res["twoshot"] and res["match"], (r, {k: v for k, v in res.items() if k != "grad_bytes"})
        assert res["buckets"] >= 2 and "twoshot" in res["bucket_routes"], res
        if mode == "reducer_ts":
            assert res["native_reducer"]
    assert out[0]["grad_bytes"] == out[1]["grad_bytes"]  # replicas identical


@gpu
def test_rccl_communicator_world1():
    from ray_lightning_accelerators_amd.parallel.comm import native_comm_module

    mod = native_comm_module()
    assert mod is not None
    c = mod.Communicator(0, 1, 0)
    c.init_rccl(mod.Communicator.unique_id())
    t = torch.arange(10, device="cuda", dtype=torch.float32)
    c.allreduce(t, 0)
    out = torch.empty(10, device="cuda")
    c.allgather(t, out)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(10, device="cuda", dtype=torch.float32)) and torch.equal(out, t)
    assert c.error_state() == 0


@gpu
def test_communicator_churn_keeps_fresh_memory_coherent():
    """Regression test for the round-5/6 intermittent corrupted-fresh-tensor failure:
    freeing hipDeviceMallocUncached memory (the communicator's xGMI / aux regions) made
    later ordinary allocations hold kernel writes the copy engine did not see
    (scripts/probes/uncached_reuse_probe.hip).  The communicator now keeps its uncached
    regions in a process-wide pool (csrc/comm/communicator.cpp uc_alloc): after many
    communicators come and go -- as in the MNIST data-parallel tests -- every fresh
    tensor written by a kernel reads the same through a kernel and through a
    device-to-host copy."""
    import gc

    from ray_lightning_accelerators_amd.ops import fused_mlp
    from ray_lightning_accelerators_amd.parallel.comm import native_comm_module

    mod = native_comm_module()
    dev = torch.device("cuda", 0)
    bad = []
    for i in range(60):
        c = mod.Communicator(0, 1, 0)
        c.aux_open([c.aux_handle(fused_mlp.mlp3_dp_capacity(32 * (1 + i % 4), 64))])
        del c
        gc.collect()
        for n in (1 << 21, (1 << 21) + (1 << 18), 136074):
            t = torch.arange(n, device=dev, dtype=torch.int32) * 3 + i  # written by a kernel
            dev_sum = int(t.long().sum())
            host_sum = int(t.cpu().long().sum())
            if dev_sum != host_sum:
                bad.append((i, n, dev_sum, host_sum))
    assert not bad, bad[:4]
