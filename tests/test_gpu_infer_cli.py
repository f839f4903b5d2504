"""GPU: infer.py end to end (reference infer.py:20-133) -- WAV chunks -> checkpoint-loaded SDDM on
the HIP device -> stitched WAVs -- and each written file equals SDDM.infer of its chunks."""
import json
import os
import struct

import numpy as np
import pytest
import torch

from _helpers import unet_config, unet_params

pytestmark = pytest.mark.gpu


def _write_pcm16(path, x, sr=16000):
    pcm = np.clip(np.round(x * 32768), -32768, 32767).astype("<i2").tobytes()
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(pcm), b"WAVE", b"fmt ", 16, 1, 1, sr, 2 * sr, 2, 16,
                      b"data", len(pcm))
    with open(path, "wb") as f:
        f.write(hdr + pcm)


def test_infer_cli_end_to_end(torch_cuda, tmp_path):
    import infer
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    from data_loader import wav_io
    from parse_config import ConfigParser
    N = 2112
    rng = np.random.default_rng(4)
    for d in ("clean", "noisy"):
        os.makedirs(tmp_path / "data" / d)
    lengths = [5000, 1000]
    for i, n in enumerate(lengths):
        c = 0.3 * np.sin(np.arange(n) * 0.05)
        _write_pcm16(tmp_path / "data" / "clean" / f"u{i}.wav", c)
        _write_pcm16(tmp_path / "data" / "noisy" / f"u{i}.wav", c + rng.uniform(-0.05, 0.05, n))
    cfg = unet_config(N, sched=("linear", 3, 1e-4, 0.05))
    cfg.update({"name": "cli", "sample_rate": 16000, "loss": "l1_loss",
                "infer_dataset": {"type": "InferDataset", "args": {"data_root": str(tmp_path / "data"),
                                                                    "datatype": ".wav"}},
                "infer_data_loader": {"type": "InferDataLoader", "args": {"batch_size": 1, "num_workers": 0}},
                "trainer": {"save_dir": str(tmp_path / "runs")}})
    # a reference-layout checkpoint of a DataParallel-trained model (module. prefix)
    diffusion = D.GaussianDiffusion("linear", 3, 1e-4, 0.05, device="cpu")
    net = NW.UNetModified2(num_samples=N, **cfg["network"]["args"])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in unet_params(N).items()})
    ref_model = M.SDDM(diffusion, net, p_transition="condition_in")
    ck = tmp_path / "model_best.pth"
    torch.save({"arch": "SDDM", "epoch": 1, "state_dict": {"module." + k: v for k, v in ref_model.state_dict().items()},
                "config": cfg}, ck)
    with open(tmp_path / "config.json", "w") as f:
        json.dump(cfg, f)
    config = ConfigParser(cfg, resume=ck, run_id="e2e")
    log = infer.main(config, seed=100)
    assert np.isfinite(log["loss"])
    ref_model = ref_model.cuda()
    for i, n in enumerate(lengths):
        out, sr = wav_io.load(os.path.join(str(config.save_dir), "samples", "output", f"u{i}.wav"))
        chunks = -(-n // N)
        assert sr == 16000 and out.shape == (1, chunks * N)
        _, noisy, _ = infer_dataset_item(tmp_path / "data", i, N)
        want = ref_model.infer(noisy.cuda(), seed=100 + i).reshape(1, -1).cpu()
        assert torch.equal(out, want)


def infer_dataset_item(root, i, N):
    from data_loader import data_loaders as DL
    return DL.InferDataset(str(root), ".wav", sample_rate=16000, T=N)[i]
