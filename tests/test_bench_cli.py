"""bench.py argument contract (the driver runs `bench.py --gpus N --steps K --warmup W`,
N > 1 under torch.distributed.run): the batch is resolved before either path runs."""
import bench


def test_default_is_config2_batch256():
    a = bench.parse_args([])
    assert (a.config, a.batch, a.gpus) == (2, 256, 1)


def test_driver_multi_gpu_args_resolve_batch():
    a = bench.parse_args(["--gpus", "8", "--steps", "50", "--warmup", "10"])
    assert a.batch == 256 and a.steps == 50 and a.warmup == 10


def test_config3_batch4096():
    assert bench.parse_args(["--config", "3"]).batch == 4096


def test_roofline_scales_out_the_instrumentation(monkeypatch):
    """The roofline's level durations come from the instrumented replay; they are scaled by
    the uninstrumented graph's time per update over the instrumented one (never up)."""
    info = dict(graph_us=2400.0, sum_us=2400.0, allreduce_us=0.0, n_updates=20, gemm_us=2000.0,
                gemm_flops=20 * 3.2e9, gemm_bytes=20 * 11 * 7.6e6, levels=220,
                kernel_launches={"k_gemm": 220}, achieved_tflops=20 * 3.2e9 / 2000e-6 / 1e12,
                sites_us={})
    monkeypatch.setattr(bench, "timeline_roofline", lambda *a, **k: dict(info))
    monkeypatch.setattr(bench, "pmc_counters", lambda *a, **k: None)
    args = bench.parse_args([])
    wl = {"dtype": "fp32"}
    r = bench.roofline_object(None, args, wl, 157.3, step_us_real=114.0)
    assert abs(r["instrumentation_scale"] - 114.0 / 120.0) < 1e-4
    assert abs(r["gemm_us_per_step"] - 100.0 * 114.0 / 120.0) < 0.01
    assert abs(r["achieved"] - 3.2e9 / (95e-6) / 1e12) < 0.01
    assert abs(r["achieved_timeline_raw"] - 32.0) < 1e-3
    r = bench.roofline_object(None, args, wl, 157.3, step_us_real=130.0)   # slower: no scaling up
    assert r["instrumentation_scale"] == 1.0 and abs(r["achieved"] - 32.0) < 1e-3


def test_pmc_figures_only_for_the_sources_they_were_measured_on(tmp_path, monkeypatch):
    import json
    import os
    monkeypatch.syspath_prepend(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import pmc_summary  # noqa: F401  (the real tools module, before ROOT moves)
    (tmp_path / "profiles").mkdir()
    z = {"csrc_digest": "0" * 16, "per_level": {"traffic_bytes": 1.0, "mfma_busy": 0.5}}
    (tmp_path / "profiles" / "pmc_c2.json").write_text(json.dumps(z))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_counters(2) is None                 # stale digest: no counters
    z["csrc_digest"] = pmc_summary.csrc_digest(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    (tmp_path / "profiles" / "pmc_c2.json").write_text(json.dumps(z))
    monkeypatch.setattr(pmc_summary, "csrc_digest", lambda root=None: z["csrc_digest"])
    assert bench.pmc_counters(2)["per_level"]["mfma_busy"] == 0.5
