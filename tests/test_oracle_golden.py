"""Pin the CPU oracle (oracle/restate.py) to golden vectors produced by the reference.

The goldens come from running the reference's own network/ package in the build
container (tests/golden/gen_golden.py). Weights are regenerated here by rpst.synth and
checked against the checksum recorded at generation time, so a generator drift fails
loudly instead of silently comparing different models.
"""
import copy
import json
import os

import numpy as np
import pytest
import torch

from helpers import (SOURCE_CONFIG, deeper_config, multiscale_config, rel_l2, rp_config,
                     state_dict_of, synth_)
from oracle import restate as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def test_stats_bitwise(golden):
    g = golden("stats")
    for i in range(int(g["n"])):
        c, s = t(g[f"c{i}"]), t(g[f"s{i}"])
        m, sd = R.calc_mean_std(c)
        np.testing.assert_array_equal(m.numpy(), g[f"cmean{i}"])
        np.testing.assert_array_equal(sd.numpy(), g[f"cstd{i}"])
        np.testing.assert_array_equal(R.adain(c, s).numpy(), g[f"adain{i}"])


def _adain_model(hidden):
    import network as net
    return net.AdaINRPNet(rp_config(hidden), copy.deepcopy(net.vgg))


def test_adain_rp_test(golden):
    g = golden("adain_rp")
    for i in range(int(g["n"])):
        m = _adain_model(int(g[f"hidden{i}"]))
        ck = synth_(m, int(g[f"seed{i}"]))
        np.testing.assert_allclose(ck, g[f"checksum{i}"], rtol=1e-12)
        sd = state_dict_of(m)
        out = R.adain_rp_test(t(g[f"content{i}"]), t(g[f"style{i}"]), sd, 5)
        assert rel_l2(out, g[f"out{i}"]) < 1e-6, i


def test_adain_rp_forward_losses(golden):
    g = golden("forward")
    m = _adain_model(4)
    np.testing.assert_allclose(synth_(m, 21), g["checksum"], rtol=1e-12)
    sd = state_dict_of(m)
    d = R.adain_rp_forward(t(g["content"]), t(g["style"]), sd, 5, 1.0, 10.0)
    for k in ("style_loss", "content_loss", "total_loss"):
        np.testing.assert_allclose(d[k].numpy(), g[k], rtol=1e-5)
    feats = R.encode_with_intermediate(t(g["content"]), sd)
    for i, f in enumerate(feats):
        assert rel_l2(f, g[f"relu{i + 1}_1"]) < 1e-6


def test_vgg_and_decoder(golden):
    import network as net
    g = golden("vgg")
    vgg = copy.deepcopy(net.vgg)
    np.testing.assert_allclose(synth_(vgg, 80), g["vgg_ck"], rtol=1e-12)
    sd = state_dict_of(vgg)
    x = t(g["x"])
    for i, (lo, hi) in enumerate(R.ENC_SLICES):
        x = R.vgg_slice(x, sd, "", lo, hi)
        assert rel_l2(x, g[f"relu{i + 1}_1"]) < 1e-6
    dec = copy.deepcopy(net.decoder)
    np.testing.assert_allclose(synth_(dec, 81), g["dec_ck"], rtol=1e-12)
    out = R.decoder(t(g["z"]), state_dict_of(dec), "")
    assert rel_l2(out, g["dec_out"]) < 1e-6


def test_wct_matrix_functions(golden):
    g = golden("wct")
    for i in range(int(g["nmat"])):
        a = t(g[f"A{i}"])
        assert rel_l2(R.matrix_sqrt(a), g[f"sqrt{i}"]) < 1e-12
        assert rel_l2(R.matrix_inv_sqrt(a), g[f"isqrt{i}"]) < 1e-12


def test_wct_whiten_and_color(golden):
    g = golden("wct")
    for i in range(int(g["ncase"])):
        out = R.whiten_and_color(t(g[f"cF{i}"]), t(g[f"sF{i}"]))
        assert rel_l2(out, g[f"wc{i}"]) < 1e-12


def _wct_large_inputs(g, i):
    from rpst import synth
    c, hw, seed = int(g[f"C{i}"]), int(g[f"HW{i}"]), int(g[f"seed{i}"])
    cf = synth.conditioned_features(seed, c, hw, 1.5)
    sf = synth.conditioned_features(seed + 50, c, hw, 3.0)
    sm = sf - sf.mean(1, keepdims=True)
    a = sm @ sm.T / (hw - 1)
    pm = 2.0 * synth.uniform01(seed, "probe", c * 8).reshape(c, 8) - 1.0
    ph = 2.0 * synth.uniform01(seed, "hwprobe", hw * 4).reshape(hw, 4) - 1.0
    return cf, sf, a, pm, ph


def test_wct_large_reference(golden):
    """C = 256 / 512 on conditioned features (reference outputs as probe products,
    gen_golden.gen_wct_large): matrix functions of the style covariance and the fused
    feature of whiten_and_color."""
    g = golden("wct_large")
    for i in range(int(g["ncase"])):
        cf, sf, a, pm, ph = _wct_large_inputs(g, i)
        assert rel_l2(R.matrix_sqrt(t(a)).numpy() @ pm, g[f"sqrtP{i}"]) < 1e-11, i
        assert rel_l2(R.matrix_inv_sqrt(t(a)).numpy() @ pm, g[f"isqrtP{i}"]) < 1e-11, i
        wc = R.whiten_and_color(t(cf), t(sf)).numpy()
        assert rel_l2(wc @ ph, g[f"wcP{i}"]) < 1e-11, i
        assert rel_l2(wc[:, :32], g[f"wcCols{i}"]) < 1e-11, i


def test_wct_edge_reference(golden):
    """The oracle's SVD form on the inputs the kernels route to the Jacobi SVD (indefinite,
    truncated, non-symmetric) and whiten_and_color at C = 512 with a dead style channel,
    against the reference (gen_golden.gen_wct_edge)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from gen_golden import wct_edge_inputs
    mats, cf, sf, ph = wct_edge_inputs()
    g = golden("wct_edge")
    for k, a in mats.items():
        assert rel_l2(R.matrix_sqrt(t(a)), g[f"sqrt_{k}"]) < 1e-12, k
        assert rel_l2(R.matrix_inv_sqrt(t(a)), g[f"isqrt_{k}"]) < 1e-12, k
    wc = R.whiten_and_color(t(cf), t(sf)).numpy()
    assert rel_l2(wc @ ph, g["wcP"]) < 1e-11 and rel_l2(wc[:, :32], g["wcCols"]) < 1e-11
    assert 5e3 < float(g["style_cov_max_eig"]) < 2e4


def test_wct_original_reference(golden):
    """whiten_and_color(method='original') (Li et al., wct_rp.py:96-101) of the oracle against
    the reference (gen_golden.gen_wct_original), including a dead style channel and C = 256."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from gen_golden import wct_original_inputs
    g = golden("wct_original")
    for i, (cf, sf, ph) in enumerate(wct_original_inputs()):
        wc = R.whiten_and_color(t(cf), t(sf), method='original').numpy()
        if ph is None:
            assert rel_l2(wc, g[f"wc{i}"]) < 1e-12, i
        else:
            assert rel_l2(wc @ ph, g[f"wcP{i}"]) < 1e-11, i
            assert rel_l2(wc[:, :32], g[f"wcCols{i}"]) < 1e-11, i


def test_wct_rp_test(golden):
    import network as net
    g = golden("wct")
    for i in range(int(g["nnet"])):
        m = net.WCTRPNet(rp_config(int(g[f"net_hidden{i}"])), copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"net_seed{i}"])), g[f"net_checksum{i}"],
                                   rtol=1e-12)
        out = R.wct_rp_test(t(g[f"net_content{i}"]), t(g[f"net_style{i}"]), state_dict_of(m), 5)
        assert rel_l2(out, g[f"net_out{i}"]) < 1e-6


def test_sanet_module_and_transform(golden):
    import network as net
    g = golden("sanet")
    for i in range(2):
        c = t(g[f"sa_c{i}"])
        mod = net.SANet(c.shape[1])
        np.testing.assert_allclose(synth_(mod, int(g[f"sa_seed{i}"])), g[f"sa_ck{i}"], rtol=1e-12)
        out = R.sanet(c, t(g[f"sa_s{i}"]), state_dict_of(mod), "")
        assert rel_l2(out, g[f"sa_out{i}"]) < 1e-6
        np.testing.assert_array_equal(R.mean_variance_norm(c).numpy(), g[f"sa_mvn{i}"])
    tr = net.Transform(32)
    np.testing.assert_allclose(synth_(tr, 60), g["tr_ck"], rtol=1e-12)
    out = R.transform(t(g["tr_c4"]), t(g["tr_s4"]), t(g["tr_c5"]), t(g["tr_s5"]),
                      state_dict_of(tr), "")
    assert rel_l2(out, g["tr_out"]) < 1e-6


def test_samodel_test(golden):
    import network as net
    g = golden("sanet")
    for i in range(2):
        c = t(g[f"model_content{i}"])
        m = net.SAModel({}, copy.deepcopy(net.vgg), 0, c.shape[-1])
        np.testing.assert_allclose(synth_(m, int(g[f"model_seed{i}"])), g[f"model_ck{i}"],
                                   rtol=1e-12)
        out = R.samodel_test(c, t(g[f"model_style{i}"]), state_dict_of(m))
        assert rel_l2(out, g[f"model_out{i}"]) < 1e-6


def test_multiscale_test(golden):
    """MultiScaleAdaINRPNet.test against the reference's outputs."""
    import network as net
    g = golden("multiscale")
    for i in range(int(g["n"])):
        hid, blocks, inc = int(g[f"hidden{i}"]), int(g[f"blocks{i}"]), int(g[f"inception{i}"])
        m = net.MultiScaleAdaINRPNet(multiscale_config(hid, blocks, inc), copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        out = R.multiscale_test(t(g[f"content{i}"]), t(g[f"style{i}"]), state_dict_of(m),
                                blocks, inc)
        assert rel_l2(out, g[f"out{i}"]) < 1e-6, (i, rel_l2(out, g[f"out{i}"]))


def test_deeper_multiscale_test(golden):
    """MultiScaleAdaINRPNet.test with enc_stack_way 'deeper' (adain_rp.py:152-156): deeper
    encoder with 1x1 inception convs, shallower decoder, against the reference's outputs."""
    import network as net
    g = golden("deeper")
    for i in range(int(g["n"])):
        hid, blocks, inc = int(g[f"hidden{i}"]), int(g[f"blocks{i}"]), int(g[f"inception{i}"])
        m = net.MultiScaleAdaINRPNet(deeper_config(hid, blocks, inc), copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        out = R.multiscale_test(t(g[f"content{i}"]), t(g[f"style{i}"]), state_dict_of(m),
                                blocks, inc)
        assert rel_l2(out, g[f"out{i}"]) < 1e-6, (i, rel_l2(out, g[f"out{i}"]))


def test_reference_training_gradients(golden):
    """The oracle's autograd gradients (R.adain_rp_grads) against the reference's own
    AdaINRPNet.forward + total_loss.backward() (adain_rp.py:110-138) gradients."""
    g = golden("grads")
    for i in range(int(g["n"])):
        m = _adain_model(int(g[f"hidden{i}"]))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        losses, grads = R.adain_rp_grads(t(g[f"content{i}"]), t(g[f"style{i}"]), state_dict_of(m),
                                         5, float(g[f"cw{i}"]), float(g[f"sw{i}"]))
        for k in ("style_loss", "content_loss", "total_loss"):
            np.testing.assert_allclose(losses[k].numpy(), g[f"{k}{i}"], rtol=1e-5)
        names = [str(n) for n in g[f"names{i}"]]
        assert sorted(names) == sorted(grads)
        for name in names:
            assert rel_l2(grads[name], g[f"grad{i}:{name}"]) < 1e-5, (i, name)


def test_reference_wct_training_gradients(golden):
    """R.wct_rp_grads against the reference's WCTRPNet.forward + backward (wct_rp.py:168-194):
    decoder gradients only (fuse() detaches the encoder features)."""
    import network as net
    g = golden("grads_wct")
    for i in range(int(g["n"])):
        m = net.WCTRPNet(rp_config(int(g[f"hidden{i}"])), copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        losses, grads = R.wct_rp_grads(t(g[f"content{i}"]), t(g[f"style{i}"]), state_dict_of(m),
                                       5, float(g[f"cw{i}"]), float(g[f"sw{i}"]))
        for k in ("style_loss", "content_loss", "total_loss"):
            np.testing.assert_allclose(losses[k].numpy(), g[f"{k}{i}"], rtol=1e-5)
        names = [str(n) for n in g[f"names{i}"]]
        assert sorted(names) == sorted(grads)
        for name in names:
            assert rel_l2(grads[name], g[f"grad{i}:{name}"]) < 1e-5, (i, name)


def test_reference_samodel_training_gradients(golden):
    """R.samodel_grads against the reference's SAModel.forward + backward
    (sanet.py:248-275): the five losses and probes of every transform / decoder gradient."""
    import network as net
    from helpers import grad_probe, probe_err
    g = golden("grads_sam")
    cfg = {"content_weight": 1.0, "style_weight": 3.0, "l_identity1_weight": 50.0,
           "l_identity2_weight": 1.0}
    for i in range(int(g["n"])):
        shp = g[f"content{i}"].shape
        m = net.SAModel(dict(cfg), copy.deepcopy(net.vgg), 0, shp[-1])
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        losses, grads = R.samodel_grads(t(g[f"content{i}"]), t(g[f"style{i}"]),
                                        state_dict_of(m), cfg)
        for k in ("style_loss", "content_loss", "l_identity1_loss", "l_identity2_loss",
                  "total_loss"):
            np.testing.assert_allclose(losses[k].numpy(), g[f"{k}{i}"], rtol=1e-5)
        names = [str(n) for n in g[f"names{i}"]]
        assert sorted(names) == sorted(grads)
        for name in names:
            e = probe_err(grad_probe(name, grads[name]), g[f"gprobe{i}:{name}"], grads[name].numel())
            assert e < 1e-5, (i, name, e)


def test_reference_adaptive_samodel_training_gradients(golden):
    """R.adaptive_samodel_grads under CPU autograd against the reference's
    AdaptiveSAModel.forward + backward (sanet.py:347-382) for both AEA modules: the losses and
    probes of every transform (incl. the f_psi MLP) and decoder gradient."""
    import network as net
    from helpers import grad_probe, probe_err
    g = golden("grads_adaptive")
    cfg = {"content_weight": 1.0, "style_weight": 3.0, "l_identity1_weight": 50.0,
           "l_identity2_weight": 1.0}
    for i in range(int(g["n"])):
        mode = str(g[f"mode{i}"])
        shp = g[f"content{i}"].shape
        m = net.AdaptiveSAModel(dict(cfg, ada_module=mode), copy.deepcopy(net.vgg), 0, shp[-1])
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        losses, grads = R.adaptive_samodel_grads(t(g[f"content{i}"]), t(g[f"style{i}"]),
                                                 state_dict_of(m), cfg, mode)
        for k in ("style_loss", "content_loss", "l_identity1_loss", "l_identity2_loss",
                  "total_loss"):
            np.testing.assert_allclose(losses[k].numpy(), g[f"{k}{i}"], rtol=1e-5)
        names = [str(n) for n in g[f"names{i}"]]
        assert sorted(names) == sorted(grads)
        for name in names:
            e = probe_err(grad_probe(name, grads[name]), g[f"gprobe{i}:{name}"], grads[name].numel())
            assert e < 1e-5, (i, name, e)


def test_reference_sourcenet_training_gradients(golden):
    """R.sourcenet_losses under CPU autograd against the reference's SourceNet.forward +
    backward (base.py:624-649): the losses and probes of every decoder gradient."""
    import network as net
    from helpers import grad_probe, probe_err, src_grads_config
    g = golden("grads_src")
    for i in range(int(g["n"])):
        cfg = src_grads_config(g, i)
        m = net.SourceNet(cfg, copy.deepcopy(net.vgg))
        m.decoder = copy.deepcopy(m.decoder)
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        losses, grads = R.grads_of(R.sourcenet_losses, state_dict_of(m), ("decoder.",),
                                   t(g[f"content{i}"]), t(g[f"style{i}"]),
                                   cfg["content_weight"], cfg["style_weight"])
        for k in ("style_loss", "content_loss", "total_loss"):
            np.testing.assert_allclose(losses[k].numpy(), g[f"{k}{i}"], rtol=1e-5)
        names = [str(n) for n in g[f"names{i}"]]
        assert sorted(names) == sorted(grads)
        for name in names:
            e = probe_err(grad_probe(name, grads[name]), g[f"gprobe{i}:{name}"], grads[name].numel())
            assert e < 1e-5, (i, name, e)


def test_reference_multiscale_training_gradients(golden):
    """R.multiscale_losses under CPU autograd against the reference's
    MultiScaleAdaINRPNet.forward + backward (adain_rp.py:321-345): constant stack with an
    inception conv, and the 'deeper' stack; every RP encoder / decoder gradient."""
    import network as net
    from helpers import ms_grads_config
    g = golden("grads_ms")
    for i in range(int(g["n"])):
        cfg = ms_grads_config(g, i)
        m = net.MultiScaleAdaINRPNet(cfg, copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        losses, grads = R.grads_of(R.multiscale_losses, state_dict_of(m),
                                   ("rp_shared_encoder.", "rp_decoder."), t(g[f"content{i}"]),
                                   t(g[f"style{i}"]), cfg["rp_blocks"], cfg["inception_num"],
                                   cfg["content_weight"], cfg["style_weight"])
        for k in ("style_loss", "content_loss", "total_loss"):
            np.testing.assert_allclose(losses[k].numpy(), g[f"{k}{i}"], rtol=1e-5)
        names = [str(n) for n in g[f"names{i}"]]
        assert sorted(names) == sorted(grads)
        for name in names:
            assert rel_l2(grads[name], g[f"grad{i}:{name}"]) < 1e-5, (i, name)


def test_sourcenet_test(golden):
    """SourceNet.test (classic AdaIN) against the reference."""
    import network as net
    g = golden("sourcenet")
    for i in range(int(g["n"])):
        m = net.SourceNet(SOURCE_CONFIG, copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        out = R.sourcenet_test(t(g[f"content{i}"]), t(g[f"style{i}"]), state_dict_of(m))
        assert rel_l2(out, g[f"out{i}"]) < 1e-6, (i, rel_l2(out, g[f"out{i}"]))


def test_adaptive_sanet_family(golden):
    """cal_affinity_matrix, AEAModule / AEALReluModule, AdaptiveSANet, AdaptiveTransform and
    AdaptiveSAModel against the reference."""
    import network as net
    g = golden("adaptive")
    aff = R.cal_affinity_matrix(t(g["aff_c"]), t(g["aff_s"]))
    assert rel_l2(aff, g["aff_out"]) < 1e-6
    for mode, cls in (("aea", net.AEAModule), ("relu", net.AEALReluModule)):
        mod = cls(48)
        np.testing.assert_allclose(synth_(mod, 90 if mode == "aea" else 91),
                                   g[f"aea_{mode}_ck"], rtol=1e-12)
        y, cl = R.aea(t(g["aff_out"]), t(g[f"aea_{mode}_fx"]), state_dict_of(mod), "", mode)
        assert rel_l2(y, g[f"aea_{mode}_out"]) < 1e-6 and rel_l2(cl, g[f"aea_{mode}_clamp"]) < 1e-6
        for i in range(2):
            c = t(g[f"asa_{mode}_c{i}"])
            mod = net.AdaptiveSANet(c.shape[1], c.shape[2] * c.shape[3], mode)
            np.testing.assert_allclose(synth_(mod, int(g[f"asa_{mode}_seed{i}"])),
                                       g[f"asa_{mode}_ck{i}"], rtol=1e-12)
            y, cl = R.adaptive_sanet(c, t(g[f"asa_{mode}_s{i}"]), state_dict_of(mod), "", mode)
            assert rel_l2(y, g[f"asa_{mode}_out{i}"]) < 1e-6, (mode, i)
            assert rel_l2(cl, g[f"asa_{mode}_claim{i}"]) < 1e-6
        tr = net.AdaptiveTransform(32, 64, 16, mode)
        np.testing.assert_allclose(synth_(tr, 98 + (mode == "relu")), g[f"atr_{mode}_ck"],
                                   rtol=1e-12)
        y = R.adaptive_transform(*(t(g[f"atr_{mode}_{k}"]) for k in ("c4", "s4", "c5", "s5")),
                                 state_dict_of(tr), "", mode)
        assert rel_l2(y, g[f"atr_{mode}_out"]) < 1e-6
        m = net.AdaptiveSAModel({"ada_module": mode}, copy.deepcopy(net.vgg), 0, 64)
        np.testing.assert_allclose(synth_(m, int(g[f"model_{mode}_seed"])), g[f"model_{mode}_ck"],
                                   rtol=1e-12)
        y = R.adaptive_samodel_test(t(g[f"model_{mode}_content"]), t(g[f"model_{mode}_style"]),
                                    state_dict_of(m), mode)
        assert rel_l2(y, g[f"model_{mode}_out"]) < 1e-6, mode


@pytest.mark.parametrize("name", ["AdaINRPNet", "WCTRPNet", "SAModel", "vgg", "decoder",
                                  "MultiScaleAdaINRPNet", "MultiScaleAdaINRPNet_inception1",
                                  "SourceNet", "AdaptiveSAModel_aea", "AdaptiveSAModel_relu"])
def test_state_dict_keys_match_reference(name):
    """Checkpoint compatibility: same keys and shapes as the reference modules."""
    import network as net
    ref = json.load(open(os.path.join(GOLD, "keys.json")))[name]
    vgg = copy.deepcopy(net.vgg)
    mine = {"AdaINRPNet": lambda: net.AdaINRPNet(rp_config(16), vgg),
            "WCTRPNet": lambda: net.WCTRPNet(rp_config(16), vgg),
            "SAModel": lambda: net.SAModel({}, vgg, 0, 512),
            "MultiScaleAdaINRPNet": lambda: net.MultiScaleAdaINRPNet(
                multiscale_config(32, 5, 0), vgg),
            "MultiScaleAdaINRPNet_inception1": lambda: net.MultiScaleAdaINRPNet(
                multiscale_config(16, 4, 1), vgg),
            "SourceNet": lambda: net.SourceNet({"use_mask": False}, vgg),
            "AdaptiveSAModel_aea": lambda: net.AdaptiveSAModel({"ada_module": "aea"}, vgg, 0,
                                                               512),
            "AdaptiveSAModel_relu": lambda: net.AdaptiveSAModel({"ada_module": "relu"}, vgg, 0,
                                                                512),
            "vgg": lambda: net.vgg, "decoder": lambda: net.decoder}[name]()
    got = [[k, list(v.shape)] for k, v in mine.state_dict().items()]
    assert got == ref
