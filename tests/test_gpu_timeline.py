"""Launch timeline of the real update graph (sacmi_profile_timeline): the instrumented
graph runs the same kernels as the timed one, the stamps are ordered, the per-kernel slots
add up to the HIP-event time of the replay, and the instrumented updates leave the model
in the same state as uninstrumented ones (the stamps change no arithmetic)."""
import numpy as np
import pytest

from oracle.sac_step import NETS, SacConfig, init_params, synthetic_rows

pytestmark = pytest.mark.gpu


def _ctx(seed=7):
    from sacmi import Config, Context
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, 5, bias_scale=0.05)
    c = Context(Config(24, 4, 64, max_batch=64, capacity=2000, seed=seed), 0)
    for n in NETS:
        c.set_net(n, params[n])
    c.push(*synthetic_rows(cfg, 2000, 6, state_scale=0.5))
    return c


def test_timeline_covers_the_update_graph():
    c = _ctx()
    ks, graph_us = c.profile_timeline(64, 4)
    names = [k["site"] for k in ks]
    # first update samples for itself, the next three ride along in L12 / L13
    assert names.count("mt_sample") == 1 and names.count("gather") == 1
    # (2 hidden layers, fp32: dL/da is folded into L9's epilogue, L10 is the sample tail)
    for site in ("gemm_L1_fc1", "gemm_L6_critic_dW_adam", "gemm_L13_pi_dW_adam", "heads_sample",
                 "gemm_L9_act_dh1", "sample_bwd_tail_dhp2"):
        assert names.count(site) == 4, site
    assert "gemm_L10_dlda_sample_bwd_dhp2" not in names
    starts = [k["start_us"] for k in ks]
    assert starts == sorted(starts)                    # graph kernels run in launch order
    assert all(k["end_us"] >= k["start_us"] for k in ks)
    span = ks[-1]["end_us"] - ks[0]["start_us"]
    assert 0 < span <= graph_us * 1.05, (span, graph_us)
    l1 = [k for k in ks if k["site"] == "gemm_L1_fc1"]
    assert all(k["kernel"] == "k_gemm" and k["flops"] > 0 and k["grid"] > 0 for k in l1)


def test_timeline_updates_equal_plain_updates():
    a, b = _ctx(), _ctx()
    a.profile_timeline(64, 3)                          # 6 instrumented updates
    b.step_many_async(64, 3)
    b.step_many_async(64, 3)
    b.synchronize()
    for n in NETS:
        pa, pb = a.get_net(n), b.get_net(n)
        for k in pa:
            assert np.array_equal(pa[k], pb[k]), (n, k)
    assert np.array_equal(a.fetch_losses(6), b.fetch_losses(6))


def test_timeline_of_the_data_parallel_sequence():
    """sacmi_profile_timeline_dp over a 1-rank communicator: the phases' kernels are
    stamped in order (plain dW levels + k_adam instead of the fused Adam levels), the
    all-reduces leave gaps before the next phase, the model ends where sacmi_step_dp
    leaves it, and bench.timeline_roofline accounts for the whole replay."""
    import bench
    from sacmi import Context
    a, b = _ctx(), _ctx()
    for c in (a, b):
        c.allreduce_init(Context.allreduce_unique_id(), 0, 1)
    ks, graph_us = a.profile_timeline(64, 3, data_parallel=True)
    names = [k["site"] for k in ks]
    assert not any(n.startswith("allreduce") for n in names)   # RCCL kernels do not stamp
    assert sum(1 for k in ks if k["kernel"] == "k_adam") == 6   # critic + actor Adam x 3
    starts = [k["start_us"] for k in ks]
    assert starts == sorted(starts)
    info = bench.timeline_roofline(a, 64, 3, data_parallel=True)
    assert info["allreduce_us"] > 0 and info["gemm_flops"] > 0
    assert abs(info["sum_us"] - info["graph_us"]) <= 0.25 * info["graph_us"], info
    for _ in range(4):                                  # 2 profiles x (warm + measured) x 3
        b.step_dp(64, 3)
    b.synchronize()
    for n in NETS:
        pa, pb = a.get_net(n), b.get_net(n)
        for k in pa:
            assert np.array_equal(pa[k], pb[k]), (n, k)


@pytest.mark.parametrize("B,x6", [(4096, True), (256, False)])
def test_fp32_level_kernels_by_batch_class(B, x6):
    """Which kernel runs each fp32 GEMM level: at batch 4096 the forward levels
    on k_fwd_x6, the dh levels (critic / actor dh1, policy dhp1) on k_axk_x6 and the weight
    gradients split-K on k_dw_part_x6 + k_dw_fin — the x6 path must be the one the batch-4096
    parity tests and bench lines exercise, not a silent k_gemm fallback; at batch 256 every
    level stays on the fp32 MFMA k_gemm."""
    from sacmi import Config, Context
    cfg = SacConfig(376, 17, 512)
    params = init_params(cfg, 11, bias_scale=0.02)
    c = Context(Config(376, 17, 512, max_batch=B, capacity=6000, seed=3), 0)
    for n in NETS:
        c.set_net(n, params[n])
    c.push(*synthetic_rows(cfg, 6000, 12, state_scale=0.1))
    ks, _ = c.profile_timeline(B, 1)
    by_site = {}
    for k in ks:
        by_site.setdefault(k["site"], []).append(k["kernel"])
    want = {"gemm_L1_fc1": ["k_fwd_x6"], "gemm_L2_fc2": ["k_fwd_x6"], "gemm_L3_tgt_fc1": ["k_fwd_x6"],
            "gemm_L4_tgt_fc2": ["k_fwd_x6"], "gemm_L7_act_fc1": ["k_fwd_x6"], "gemm_L8_act_fc2": ["k_fwd_x6"],
            "gemm_L5_critic_dh1": ["k_axk_x6"], "gemm_L9_act_dh1": ["k_axk_x6"], "gemm_L12_pi_dhp1": ["k_axk_x6"],
            "gemm_L6_critic_dW_adam": ["k_dw_part_x6", "k_dw_fin"],
            "gemm_L13_pi_dW_adam": ["k_dw_part_x6", "k_dw_fin"]}
    for site, kernels in want.items():
        got = by_site.get(site)
        assert got, (site, sorted(by_site))
        if x6:
            assert got == kernels, (site, got)
        else:
            assert got == ["k_gemm"], (site, got)
    c.close()
