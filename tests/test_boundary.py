"""Drop-in boundary (CPU): the C-ABI library loads and exports every declared symbol, its host-only
schedule code matches the reference, and the facade mirrors the reference's plugin surface
(module paths, class names, kwargs, state_dict layout, error types).  No GPU calls."""
import json
import os
import re

import numpy as np
import pytest
import torch

import sddm_hip
from _helpers import GOLDEN, UNET_NET, parse_sched_key, tables_from_golden
from oracle.schedule import BUFFER_NAMES

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "sddm_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sddm_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = sddm_hip.lib()
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(sddm_hip.EXPORTS)
    assert lib.sddm_abi_version() == 1


@pytest.mark.parametrize("key", ["linear_1000_1e-06_0.001", "linear_200_0.0001_0.02", "quad_100_0.0001_0.02",
                                 "cosine_1000_0.0001_0.02", "linear_50_0.0001_0.05"])
def test_library_schedule_matches_reference(key):
    ref = tables_from_golden(key)
    got = sddm_hip.schedule(*parse_sched_key(key))
    for k in BUFFER_NAMES:
        r, g = ref[k], got[k]
        assert np.array_equal(np.isnan(r), np.isnan(g)), k
        ok = ~np.isnan(r)
        if not key.startswith("cosine") and k in ("betas", "alphas", "alpha_bar"):
            assert np.array_equal(r.view(np.uint32), g.view(np.uint32)), k
        else:
            rel = np.abs(r[ok] - g[ok]) / np.maximum(np.abs(r[ok]), 1e-3)
            assert rel.max() <= 2e-2, (k, rel.max())


def test_library_schedule_unknown_raises():
    with pytest.raises(NotImplementedError):
        sddm_hip.schedule("warmup10", 10, 1e-4, 0.02)


def _build(num_samples=2112, p_transition="condition_in"):
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    d = D.GaussianDiffusion("linear", 100, 1e-6, 1e-3, device="cpu")
    n = NW.UNetModified2(num_samples=num_samples, **UNET_NET["args"])
    return M.SDDM(d, n, p_transition=p_transition)


def test_facade_state_dict_matches_reference_layout():
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))["unet_2112_T100"]
    mine = [[k, list(v.shape)] for k, v in _build().state_dict().items()]
    assert mine == ref


def test_facade_buffers_equal_library_schedule():
    m = _build()
    got = sddm_hip.schedule("linear", 100, 1e-6, 1e-3)
    for k in BUFFER_NAMES:
        assert np.array_equal(getattr(m.diffusion, k).numpy(), got[k], equal_nan=True)


def test_facade_load_state_dict_roundtrip():
    m = _build()
    sd = {k: torch.randn_like(v) if v.dtype.is_floating_point else v for k, v in m.state_dict().items()}
    m2 = _build()
    m2.load_state_dict(sd)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k])


def test_facade_rejects_unknown_modes_like_reference():
    with pytest.raises(NotImplementedError):
        _build(p_transition="ddim")
    import model.diffusion as D
    with pytest.raises(NotImplementedError):
        D.GaussianDiffusion("warmup10", 10, device="cpu")
    import model.model as M
    with pytest.raises(NotImplementedError):
        M.SDDM(D.GaussianDiffusion("linear", 10, device="cpu"), torch.nn.Identity(), noise_condition="snr")


def test_training_forward_needs_the_hip_device():
    """SDDM.forward (model.py:29-48) runs q-sample + network on HIP; host tensors raise, never a
    silent CPU fallback."""
    m = _build()
    x = torch.zeros(1, 1, 2112)
    with torch.no_grad(), pytest.raises(RuntimeError) as e:
        m(x, x)
    assert not isinstance(e.value, NotImplementedError)


def test_training_forward_refuses_autograd():
    """The HIP training-step forward has no backward: in grad mode with trainable parameters (the
    reference's Trainer._train_epoch, trainer.py:64-73) it raises NotImplementedError up front
    instead of returning tensors that fail later at loss.backward()."""
    m = _build()
    x = torch.zeros(1, 1, 2112)
    with pytest.raises(NotImplementedError):
        m(x, x)
    for p in m.parameters():
        p.requires_grad_(False)
    with pytest.raises(RuntimeError) as e:          # past the autograd check: host tensors refused
        m(x, x)
    assert not isinstance(e.value, NotImplementedError)


def test_facade_geometry_assert_like_reference():
    import model.network as NW
    with pytest.raises(AssertionError):
        NW.UNetModified2(num_samples=2100, **UNET_NET["args"])   # (2100-128) % 64 != 0 (UNetModified2.py:13)


def test_facade_requires_hip_device_no_cpu_fallback():
    m = _build()
    with pytest.raises(RuntimeError):
        m.infer(torch.zeros(1, 1, 2112))


def test_config_parser_init_obj_resolves_plugins(tmp_path):
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.model as module_arch
    import model.network as module_network
    cfg = read_json(os.path.join(REPO, "speech-denoising-diffusion-model-2_amd", "configs", "config_unet_bench.json"))
    cfg["trainer"] = {"save_dir": str(tmp_path)}
    config = ConfigParser(cfg, run_id="t")
    assert (tmp_path / cfg["name"] / "t" / "config.json").exists()
    diffusion = config.init_obj("diffusion", module_diffusion, device="cpu")
    network = config.init_obj("network", module_network, num_samples=config["num_samples"])
    model = config.init_obj("arch", module_arch, diffusion, network)
    assert type(model).__name__ == "SDDM" and model.p_transition == "condition_in"
    assert model.num_timesteps == 1000 and len(model.state_dict()) == 232 + 0
    with pytest.raises(AssertionError):
        config.init_obj("network", module_network, num_samples=1, in_channel=2)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference configs only in the build container")
@pytest.mark.parametrize("name", ["config_unet.json"])
def test_reference_config_resolves_unchanged(name, tmp_path):
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.model as module_arch
    import model.network as module_network
    cfg = read_json(os.path.join("/root/reference", name))
    cfg["trainer"]["save_dir"] = str(tmp_path)
    config = ConfigParser(cfg, run_id="r")
    diffusion = config.init_obj("diffusion", module_diffusion, device="cpu")
    network = config.init_obj("network", module_network, num_samples=config["num_samples"])
    model = config.init_obj("arch", module_arch, diffusion, network)
    lib_cfg = model.library_config()
    assert lib_cfg["network"]["args"]["channel_mults"] == [1, 2, 3, 4, 5]
    assert lib_cfg["arch"]["args"]["p_transition"] == "condition_in"


def test_wavegrad_facade_state_dict_matches_reference_layout():
    import model.network as NW
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_keys.json")))["wavegrad"]
    sd = NW.WaveGrad().state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == ref


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference configs only in the build container")
def test_reference_wavegrad_config_resolves_unchanged(tmp_path):
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.model as module_arch
    import model.network as module_network
    cfg = read_json(os.path.join("/root/reference", "config_wavegrad.json"))
    cfg["trainer"]["save_dir"] = str(tmp_path)
    config = ConfigParser(cfg, run_id="w")
    diffusion = config.init_obj("diffusion", module_diffusion, device="cpu")
    network = config.init_obj("network", module_network, num_samples=-1)
    model = config.init_obj("arch", module_arch, diffusion, network)
    lib_cfg = model.library_config()
    assert type(model).__name__ == "SDDM_spectrogram" and model.hop_samples == 300
    assert lib_cfg["network"]["type"] == "WaveGrad" and lib_cfg["diffusion"]["args"]["n_timestep"] == 1000


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference configs only in the build container")
@pytest.mark.parametrize("name,net,hop,bins", [("config_diffwave.json", "DiffWave", 256, 513),
                                               ("config_wavegrad.json", "WaveGrad", 300, 128),
                                               ("config_unet.json", "UNetModified2", None, None)])
def test_reference_configs_build_unchanged(name, net, hop, bins, tmp_path):
    """model.build_from_config resolves the reference JSONs as they are: config_diffwave.json names
    its bins 'stft_bins'  and gives the arch no hop_samples (Q6); both come from its
    'spectrogram' section, as train_specmodel.py:21-49 derives them."""
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.model as module_arch
    import model.network as module_network
    cfg = read_json(os.path.join("/root/reference", name))
    cfg["trainer"]["save_dir"] = str(tmp_path)
    config = ConfigParser(cfg, run_id="b")
    diffusion, network, model = module_arch.build_from_config(config, module_diffusion, module_network,
                                                              module_arch, "cpu")
    assert type(network).__name__ == net
    if hop is not None:
        assert type(model).__name__ == "SDDM_spectrogram" and model.hop_samples == hop
        assert network.freq_bins == bins
    lib = model.library_config()
    assert lib["network"]["type"] == net
    assert lib["diffusion"]["args"]["n_timestep"] == cfg["diffusion"]["args"]["n_timestep"]
