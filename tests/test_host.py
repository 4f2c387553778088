"""Host-side logic that runs without a GPU: parameter spec, arena layout, FLOP model,
synthetic data contract."""
import numpy as np
import torch

from optical_flow_amd import params as P


def test_param_count_and_layout():
    spec = P.flow_net_spec()
    train = [p for p in spec if p.trainable]
    assert sum(p.size for p in train) == 4938760            # 4.94 M params
    assert P.head_cin(0) == 305 and P.head_cin(1) == 179 and P.head_cin(3) == 115
    names = [p.name for p in spec]
    assert len(names) == len(set(names))
    blocks = list(P.encoder_blocks())
    assert [b[3] for b in blocks] == [1, 1, 2, 1, 2, 1]
    assert [b[4] for b in blocks] == [False, False, True, False, True, False]


def test_stage_blocks_match_encoder():
    """resnet_layer_simple's stage layout (model.py:18,20,22) composes into the encoder's."""
    stages = (P.stage_blocks(2, 64, 2, False) + P.stage_blocks(3, 64, 2, True) +
              P.stage_blocks(4, 128, 2, True))
    assert stages == list(P.encoder_blocks())
    assert P.blocks_spec(stages) == P.encoder_spec()[6:]     # after conv1 + layer1_bn
    s = P.stage_blocks(4, 128, 3, False)                    # channel change, no downsample
    assert [(b[3], b[4]) for b in s] == [(1, True), (1, False), (1, False)]
    assert s[-1][0] == "ResNet18/res4_2" and s[0][2] == 256


def test_glorot_init_deterministic():
    a = P.init_params(P.head_spec(3), 0)
    b = P.init_params(P.head_spec(3), 0)
    for k in a:
        assert np.array_equal(a[k], b[k])
    k = a["flow_module_3/conv0/kernel"]
    limit = np.sqrt(6.0 / (9 * 115 + 9 * 128))
    assert k.min() >= -limit and k.max() <= limit
    assert not a["flow_module_3/conv0/bias"].any()


def test_param_store_arena_cpu():
    from optical_flow_amd.model import ParamStore, backward_order
    order = backward_order()
    spec = P.flow_net_spec()
    assert sorted(order) == sorted(p.name for p in spec if p.trainable)
    st = ParamStore(spec, device="cpu", order=order)
    assert st.arena_order[0].startswith("flow_module_3/")       # finest head first
    assert st.arena_order[-1] == "ResNet18/conv1/kernel"         # stem last
    for name, off in st.offsets.items():
        assert off % 4 == 0                                      # 16-byte aligned views
        assert st.params[name].data_ptr() == st.arena.data_ptr() + 4 * off
        assert st.params[name]._of_grad.data_ptr() == st.grad_arena.data_ptr() + 4 * off
    vals = P.init_params(spec, 0)
    for k, v in vals.items():
        assert np.array_equal(st.params[k].detach().numpy(), v)


def test_flop_model_matches_survey():
    import bench
    assert abs(bench.gflop_per_pair(384, 512) - 249.8) < 0.1
    assert abs(bench.gflop_per_pair(128, 256) - 41.6) < 0.1
    assert abs(bench.gflop_per_pair(768, 1024) - 999.4) < 0.1


def test_synthetic_value_contract():
    from optical_flow_amd.data import IMAGE_MEANS, synthetic_batch
    b = synthetic_batch(2, 32, 48, seed=3)
    assert b.shape == (2, 32, 48, 6) and b.dtype == np.float32
    assert b.min() > -IMAGE_MEANS.max() - 0.1 and b.max() < 1.0 - IMAGE_MEANS.min() + 0.1
    assert np.array_equal(b, synthetic_batch(2, 32, 48, seed=3))
    assert not np.array_equal(b, synthetic_batch(2, 32, 48, seed=3, rank=1))


def test_five_level_spec():
    """levels=5 adds encoder stage 5 (512 ch, H/32) and a fifth flow head (model.py:24-25)."""
    from optical_flow_amd import params as P
    assert P.head_cin(0, levels=5) == 512 + 49
    assert P.head_cin(1, levels=5) == 256 + 49 + 2 and P.head_cin(4, levels=5) == 64 + 49 + 2
    blocks = list(P.encoder_blocks(5))
    assert len(blocks) == 8 and blocks[-2][2] == 512 and blocks[-2][3] == 2 and blocks[-2][4]
    names = {p.name for p in P.flow_net_spec(levels=5)}
    assert "flow_module_4/conv5/kernel" in names and "ResNet18/res5_1/conv_b/kernel" in names
    assert "flow_module_4/conv0/kernel" not in {p.name for p in P.flow_net_spec()}


def test_bench_kernel_symbols_match_pmc_keys():
    """bench.py names each split-kernel timing kind by its demangled rocprofv3 symbol (the
    defaulted NB template argument included); every x3 instance that the committed PMC pass
    saw must be reachable from a kind, or roofline.traffic silently comes out null."""
    import json
    import os
    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    entries = json.load(open(os.path.join(root, "profiles", "pmc_traffic.json")))["entries"]
    keys = set().union(*(e["kernels"] for e in entries.values()))
    names = set()
    for mode in (0, 1):
        for cfg in bench.X3_BN:
            names.add(bench.kernel_symbol(128 + mode * 8 + cfg))
    for cfg in bench.X3_WGT:
        names.add(bench.kernel_symbol(128 + 16 + cfg if cfg < 8 else 152 + cfg - 8))
    for mode in (0, 1):
        for cfg in bench.GX3:
            names.add(bench.kernel_symbol(160 + mode * 8 + cfg))
    for cfg in bench.GX3_WG:
        names.add(bench.kernel_symbol(176 + cfg))
    for mode in (0, 1):                      # the one-plane (bf16) split GEMMs
        for cfg in bench.GX3:
            names.add(bench.kernel_symbol(240 + mode * 8 + cfg))
    for cfg in bench.GX3_WG:
        names.add(bench.kernel_symbol(256 + cfg))
    for kind in (bench.KIND_STEM_X3, bench.KIND_STEM_WG_X3, bench.KIND_STEM_B16,
                 bench.KIND_STEM_WG_B16):
        names.add(bench.kernel_symbol(kind))
    x3_keys = {k for k in keys if "_x3<" in k or "_x3b<" in k}
    assert x3_keys and x3_keys <= names, sorted(x3_keys - names)
    # the bf16 image kernels (conv_b16i.hip; their template also carries the persistent flag)
    b16i = set()
    for mode in (0, 1):
        for cfg in bench.HALO_B16:
            b16i.add(bench.kernel_symbol(288 + mode * 8 + cfg))
    for cfg in bench.WGRAD_B16I:
        b16i.add(bench.kernel_symbol(304 + cfg))
    b16i_keys = {k for k in keys if "conv_halo_b16<" in k or "conv_wgrad_b16i<" in k}
    assert b16i_keys and b16i_keys <= b16i, sorted(b16i_keys - b16i)


def test_draw_all_arrows_geometry():
    """drawing.py:17-34 arrow grid: 8 rows x 15 columns of anchors, the tip at the rounded,
    clamped displaced point, the blend (img1 + img2) / 2 elsewhere."""
    from optical_flow_amd.drawing import ARROW_COLOR, _arrow_anchors, _arrow_end, draw_all_arrows
    h, w = 32, 60
    img1 = np.full((h, w, 3), 0.2, np.float32)
    img2 = np.full((h, w, 3), 0.6, np.float32)
    flow = np.zeros((h, w, 2), np.float32)
    flow[..., 0] = 2.5                       # rounds half-to-even: tip at x + 2
    flow[..., 1] = 100.0                     # clamped to the last row
    pic = draw_all_arrows(img1, img2, flow)
    anchors = _arrow_anchors(h, w)
    assert len(anchors) == 8 * 15 and anchors[0] == (0, 0) and anchors[-1] == (56, 28)
    assert _arrow_end(4, 8, flow[8, 4], w, h) == (6, h - 1)
    assert _arrow_end(58, 0, (5.0, -3.0), w, h) == (w - 1, 0)
    for x, y in anchors:
        tx, ty = _arrow_end(x, y, flow[y, x], w, h)
        np.testing.assert_array_equal(pic[ty, tx], ARROW_COLOR)
    untouched = pic[(pic != np.array(ARROW_COLOR, np.float32)).any(-1)]
    np.testing.assert_allclose(untouched, 0.4, rtol=1e-6)


def test_flowgrad_release_deferred_to_join():
    """inside a backward that forked side streams, a flow head's loss-gradient
    buffer may still be read there by the head's weight gradient; FlowGrad.release then
    pools it only at the end-of-backward join (ops._side_join), after the current stream has
    been ordered behind the side streams, so the next FlowGrad cannot pop and overwrite it
    first.  Without side streams armed it is pooled at once."""
    from optical_flow_amd import ops
    key_shape = (1, 3, 5, 2)
    ops.FlowGrad._pool.pop(("cpu", key_shape), None)
    fg = ops.FlowGrad(key_shape, "cpu")
    buf = fg.buffer()
    prev = ops._side_armed
    try:
        ops._side_armed = True
        fg.release()
        assert not ops.FlowGrad._pool.get(("cpu", key_shape))
        other = ops.FlowGrad(key_shape, "cpu")
        assert other.buffer() is not buf          # not handed out before the join
        ops._side_join()
        assert ops.FlowGrad._pool[("cpu", key_shape)][-1] is buf
        ops._side_armed = False
        other.release()
        assert len(ops.FlowGrad._pool[("cpu", key_shape)]) == 2     # pooled at once
    finally:
        ops._side_armed = prev
        ops.FlowGrad._pool.pop(("cpu", key_shape), None)
