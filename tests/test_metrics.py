"""Observability: ThroughputMonitor (cross-rank step-time aggregation) and the
Prometheus exporter."""
import urllib.request

import ray_lightning_accelerators_amd.lightning as pl
from ray_lightning_accelerators_amd.models.boring import BoringModel
from ray_lightning_accelerators_amd.utils.metrics import PrometheusExporter, ThroughputMonitor, metric_name


def test_metric_name_sanitised():
    assert metric_name("ptl/val_loss") == "rla_ptl_val_loss"
    assert metric_name("perf/step_ms_p99") == "rla_perf_step_ms_p99"


def test_throughput_monitor_and_prometheus_exporter(tmpdir):
    mon = ThroughputMonitor()
    exp = PrometheusExporter(port=0, every_n_steps=2)
    trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=2, limit_train_batches=6, limit_val_batches=2,
                         callbacks=[mon, exp], checkpoint_callback=False)
    try:
        assert trainer.fit(BoringModel()) == 1
        assert len(mon.history) == 2
        h = mon.history[-1]
        assert h["ranks"] == 1 and h["samples_per_sec"] > 0 and h["step_ms_p99"] >= h["step_ms_p50"] > 0
        assert float(trainer.callback_metrics["perf/samples_per_sec"]) > 0
        body = urllib.request.urlopen(f"http://127.0.0.1:{exp.port}/metrics", timeout=10).read().decode()
        assert "rla_perf_samples_per_sec" in body and "rla_global_step" in body
        assert "rla_val_loss" in body  # BoringModel logs val_loss
    finally:
        exp.close()


def test_exporter_pickles_without_server():
    import cloudpickle

    exp = PrometheusExporter(port=0)
    exp.on_fit_start(type("T", (), {"global_rank": 0, "global_step": 0})(), None)
    try:
        clone = cloudpickle.loads(cloudpickle.dumps(exp))
        assert clone._server is None and clone.port == exp.port
    finally:
        exp.close()


class _CheckAggregated(ThroughputMonitor):
    """Runs inside the workers: the epoch summary must cover both ranks."""

    def on_train_epoch_end(self, trainer, pl_module, outputs=None):
        super().on_train_epoch_end(trainer, pl_module, outputs)
        h = self.history[-1]
        assert h["ranks"] == 2 and h["samples_per_sec"] > 0, h
        assert h["straggler_rank"] in (0.0, 1.0)


def test_throughput_monitor_aggregates_across_workers(tmpdir):
    from ray_lightning_accelerators_amd import RayAccelerator
    from ray_lightning_accelerators_amd import runtime as ray

    ray.init(num_cpus=2, num_gpus=0)
    try:
        trainer = pl.Trainer(default_root_dir=str(tmpdir), max_epochs=1, limit_train_batches=4,
                             limit_val_batches=1, callbacks=[_CheckAggregated()], checkpoint_callback=False,
                             accelerator=RayAccelerator(num_workers=2))
        assert trainer.fit(BoringModel()) == 1
    finally:
        ray.shutdown()
