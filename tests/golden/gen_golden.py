"""Generate golden vectors by running the REFERENCE Python on CPU (build container only).

Usage (from the repo root, with the reference mounted read-only):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [--reference /root/reference]

The reference is imported read-only; its modules are built with the
deterministic weights of ``tests/_weights.py`` and ``torch.randn_like`` /
``torch.randn`` are replaced by the counter-based stream of ``oracle.philox``
(draw 0 = x_T, draw t = transition noise at step t), exactly the stream the
HIP kernels generate.  Only inputs and outputs are written (``*.npz`` data
fixtures, no reference source); the reference never travels to the GPU box.
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

SCHEDULES = [("linear", 4, 1e-6, 1e-3), ("linear", 50, 1e-6, 1e-3), ("linear", 100, 1e-6, 1e-3),
             ("linear", 1000, 1e-6, 1e-3), ("linear", 200, 1e-4, 0.02), ("linear", 1000, 1e-6, 0.01),
             ("linear", 50, 1e-4, 0.05), ("quad", 100, 1e-4, 0.02), ("cosine", 100, 1e-4, 0.02),
             ("cosine", 1000, 1e-4, 0.02), ("linear", 3, 1e-4, 0.05)]
UNET_ARGS = dict(in_channel=2, out_channel=1, inner_channel=32, norm_groups=32,
                 channel_mults=[1, 2, 3, 4, 5], res_blocks=1, dropout=0, segment_len=128,
                 segment_stride=64)   # config_unet.json "network.args"


def sched_key(s):
    return f"{s[0]}_{s[1]}_{s[2]:g}_{s[3]:g}"


class NoiseInjector:
    """Replaces torch.randn_like / torch.randn with the Philox stream."""

    def __init__(self, torch, philox, seed):
        self.torch, self.philox, self.seed = torch, philox, seed
        self.draws = []

    def __enter__(self):
        t = self.torch
        self._rl, self._r = t.randn_like, t.randn

        def randn_like(x, *a, **kw):
            d = self.draws.pop(0)
            return t.from_numpy(self.philox.normal(self.seed, d, tuple(x.shape)))

        def randn(*shape, **kw):
            if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
                shape = tuple(shape[0])
            d = self.draws.pop(0)
            return t.from_numpy(self.philox.normal(self.seed, d, tuple(int(s) for s in shape)))

        t.randn_like, t.randn = randn_like, randn
        return self

    def __exit__(self, *exc):
        self.torch.randn_like, self.torch.randn = self._rl, self._r
        assert not self.draws, f"unused draws {self.draws}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default=None, help="regenerate one fixture group (stft, q, wavegrad, long, torchnoise)")
    args = ap.parse_args()
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "speech-denoising-diffusion-model-2_amd"))
    if args.only == "stft":               # torch.stft restatement only: nothing from the reference
        import torch
        gen_stft(torch, args.out)
        return
    sys.path.insert(0, args.reference)
    import torch
    torch.set_num_threads(8)
    from oracle import philox
    from oracle.unet import architecture
    from sddm_hip.synth import noisy_speech
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _weights import make_params
    from model.diffusion import GaussianDiffusion
    from model.UNetModified2 import UNetModified2, PositionalEncoding
    from model.model import SDDM
    out = {}
    if args.only == "q":
        gen_q(torch, GaussianDiffusion, args.out)
        return
    if args.only == "wavegrad":
        gen_wavegrad(torch, philox, make_params, GaussianDiffusion, args.out)
        return
    if args.only == "long":
        gen_long(torch, philox, make_params, GaussianDiffusion, noisy_speech, args.out)
        return
    if args.only == "torchnoise":
        gen_torchnoise(torch, make_params, GaussianDiffusion, noisy_speech, args.out)
        return

    # 1. schedule tables (diffusion.py:50-161)
    for s in SCHEDULES:
        d = GaussianDiffusion(*s, device="cpu")
        for k, v in d.state_dict().items():
            out[f"sched/{sched_key(s)}/{k}"] = v.numpy().copy()
    np.savez_compressed(os.path.join(args.out, "schedules.npz"), **out)

    # 2. embedding vector (UNetModified2.py:53-55)
    emb = {"unet_embedding_vector": PositionalEncoding(32).embedding_vector.numpy().copy()}

    def build_unet(n_samples, sched, mode="condition_in", seed=0):
        d = GaussianDiffusion(*sched, device="cpu")
        net = UNetModified2(num_samples=n_samples, **UNET_ARGS)
        m = SDDM(d, net, p_transition=mode)
        shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
        P = make_params(shapes, seed)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
        m.eval()
        return m, d, net

    # 3. state-dict key layout of the three configs (boundary contract)
    m, _, _ = build_unet(2112, SCHEDULES[2])
    keys = {"unet_2112_T100": [[k, list(v.shape)] for k, v in m.state_dict().items()]}
    with open(os.path.join(args.out, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)

    # 4. transitions, each mode, at a few t (diffusion.py:164-223)
    tr = {}
    rng = np.random.default_rng(42)
    for s in (SCHEDULES[2], SCHEDULES[4]):
        d = GaussianDiffusion(*s, device="cpu")
        T = s[1]
        for mode in ("original", "sr3", "supportive", "conditional"):
            for t in (T, T // 2, 2, 1):
                x_t = rng.uniform(-1, 1, (2, 1, 256)).astype(np.float32)
                eps = rng.standard_normal((2, 1, 256)).astype(np.float32)
                cond = rng.uniform(-1, 1, (2, 1, 256)).astype(np.float32)
                key = f"tr/{sched_key(s)}/{mode}/{t}"
                inj = NoiseInjector(torch, philox, 7)
                inj.draws = [t] if t > 1 else []
                with inj:
                    X, E, C = map(torch.from_numpy, (x_t, eps, cond))
                    if mode == "original":
                        y = d.p_transition(X, t, E)
                    elif mode == "sr3":
                        y = d.p_transition_sr3(X, t, E)
                    elif mode == "supportive":
                        y = d.p_transition_supportive(X, t, E, C)
                    else:
                        y = d.p_transition_conditional(X, t, E, C)
                tr[key + "/x_t"], tr[key + "/eps"], tr[key + "/cond"] = x_t, eps, cond
                tr[key + "/out"] = y.numpy().copy()
        # get_x_T variants (diffusion.py:281-320)
        cond = rng.uniform(-1, 1, (2, 1, 256)).astype(np.float32)
        for name in ("get_x_T", "get_x_T_conditional"):
            inj = NoiseInjector(torch, philox, 7)
            inj.draws = [0]
            with inj:
                y = getattr(d, name)(torch.from_numpy(cond))
            tr[f"tr/{sched_key(s)}/{name}/cond"] = cond
            tr[f"tr/{sched_key(s)}/{name}/out"] = y.numpy().copy()
    np.savez_compressed(os.path.join(args.out, "transitions.npz"), **tr)

    # 5. UNet single forward (UNetModified2.py:237-269)
    fw = {}
    for N, B in ((2112, 2), (16448, 1)):
        m, d, net = build_unet(N, SCHEDULES[2])
        cond = noisy_speech(B, N, seed=1234)
        x_t = philox.normal(11, 0, (B, 1, N))
        nl = np.array([0.93, 0.41][:B], dtype=np.float32).reshape(B, 1, 1)
        with torch.no_grad():
            y = net(torch.from_numpy(cond), torch.from_numpy(x_t), torch.from_numpy(nl))
        fw[f"fw/{N}/cond"], fw[f"fw/{N}/x_t"], fw[f"fw/{N}/noise_level"] = cond, x_t, nl.reshape(-1)
        fw[f"fw/{N}/eps"] = y.numpy().copy()
    np.savez_compressed(os.path.join(args.out, "unet_forward.npz"), **fw)

    # 6. full SDDM.infer loops (model.py:50-124) with the Philox stream, every mode
    inf = {}
    for mode, sched, N, B in (("condition_in", SCHEDULES[0], 2112, 2), ("original", SCHEDULES[10], 2112, 2),
                              ("sr3", SCHEDULES[10], 2112, 1), ("supportive", SCHEDULES[10], 2112, 1),
                              ("conditional", SCHEDULES[10], 2112, 1),
                              ("condition_in", SCHEDULES[1], 16448, 1)):
        m, d, net = build_unet(N, sched, mode)
        T = sched[1]
        cond = noisy_speech(B, N, seed=1234)
        steps = []
        orig = d.p_transition, d.p_transition_sr3, d.p_transition_supportive, d.p_transition_conditional

        def rec(fn):
            def w(*a, **kw):
                y = fn(*a, **kw)
                steps.append(y.numpy().copy())
                return y
            return w
        d.p_transition, d.p_transition_sr3, d.p_transition_supportive, d.p_transition_conditional = map(rec, orig)
        inj = NoiseInjector(torch, philox, 7)
        inj.draws = ([] if mode == "supportive" else [0]) + list(range(T, 1, -1))
        with inj, torch.no_grad():
            y = m.infer(torch.from_numpy(cond))
        key = f"inf/{mode}/{sched_key(sched)}/{N}x{B}"
        inf[key + "/cond"] = cond
        inf[key + "/out"] = y.numpy().copy()
        if N <= 2112:
            inf[key + "/steps"] = np.stack(steps)
    np.savez_compressed(os.path.join(args.out, "unet_infer.npz"), **inf)

    # 7. DiffWave (model/diffwave.py) forward and SDDM_spectrogram.infer (model.py:212-257)
    #    config_diffwave.json network args; spectrogram [B, 513, F] ~ U[0, 1]
    from model.diffwave import DiffWave, DiffusionEmbedding
    from model.model import SDDM_spectrogram
    emb["diffwave_embedding_vector"] = DiffusionEmbedding().embedding_vector.numpy().copy()
    dw = {}
    rng = np.random.default_rng(5)
    for F, B in ((6, 2),):
        net = DiffWave(num_samples=-1, num_timesteps=3, freq_bins=513, residual_channels=64,
                       residual_layers=30, dilation_cycle_length=10)
        shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
        P = make_params(shapes, 0)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
        net.eval()
        spec = rng.uniform(0, 1, (B, 513, F)).astype(np.float32)
        N = 256 * F
        audio = philox.normal(13, 0, (B, 1, N))
        steps = np.array([3.0, 1.0][:B], dtype=np.float32).reshape(B, 1, 1)
        with torch.no_grad():
            y = net(torch.from_numpy(spec), torch.from_numpy(audio), torch.from_numpy(steps))
            up = net.spectrogram_upsampler(torch.from_numpy(spec))
        key = f"dw/fw/{F}x{B}"
        dw[key + "/spec"], dw[key + "/audio"], dw[key + "/step"] = spec, audio, steps.reshape(-1)
        dw[key + "/eps"] = y.numpy().copy()
        dw[key + "/upsampled"] = up.numpy()[:, :64].copy()   # first 64 bins (fixture size)
        # full sampling loop, time_step conditioning (config_diffwave.json arch args)
        sched = SCHEDULES[10]
        d = GaussianDiffusion(*sched, device="cpu")
        m = SDDM_spectrogram(d, net, hop_samples=256, noise_condition="time_step")
        m.eval()
        steps_rec = []
        orig = d.p_transition

        def rec(*a, **kw):
            y = orig(*a, **kw)
            steps_rec.append(y.numpy().copy())
            return y
        d.p_transition = rec
        inj = NoiseInjector(torch, philox, 7)
        inj.draws = [0] + list(range(sched[1], 1, -1))
        with inj, torch.no_grad():
            y = m.infer(torch.from_numpy(spec))
        key = f"dw/inf/time_step/{sched_key(sched)}/{F}x{B}"
        dw[key + "/spec"] = spec
        dw[key + "/out"] = y.numpy().copy()
        dw[key + "/steps"] = np.stack(steps_rec)
    keys["diffwave_513"] = [[k, list(v.shape)] for k, v in net.state_dict().items()]
    with open(os.path.join(args.out, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)
    np.savez_compressed(os.path.join(args.out, "diffwave.npz"), **dw)
    np.savez_compressed(os.path.join(args.out, "embedding.npz"), **emb)
    gen_wavegrad(torch, philox, make_params, GaussianDiffusion, args.out)
    gen_q(torch, GaussianDiffusion, args.out)
    gen_stft(torch, args.out)
    print("wrote fixtures to", args.out)


def gen_stft(torch, out_dir):
    """10. prepare_spectrogram.py:20-55 features.  torchaudio is absent, so the fixture restates
    torchaudio.functional.spectrogram with torch.stft (center, reflect, onesided, 'window'
    normalisation, power 1) and MelScale with the facade's melscale_fbanks (torch fp32 ops)."""
    from features import melscale_fbanks
    from sddm_hip.synth import noisy_speech
    st = {}
    audio = noisy_speech(2, 4000, seed=3).reshape(2, -1).astype(np.float32)
    audio[1, 1000:1400] = 0.0                                      # exact-zero stretch (log10(0) edge)
    x = torch.from_numpy(audio)

    def magnitude(w):
        spec = torch.stft(x, 1024, 256, 1024, w, center=True, pad_mode="reflect", normalized=False, onesided=True,
                          return_complex=True)
        return (spec / w.pow(2.).sum().sqrt()).abs()

    w = torch.hamming_window(1024)                 # Spectrogram(window_fn=torch.hamming_window)
    wm = torch.hann_window(1024)                   # MelSpectrogram: no window_fn -> torchaudio's Hann
    mag = magnitude(w)
    fb = melscale_fbanks(513, 20.0, 8000.0, 128, 16000)
    mel = torch.matmul(magnitude(wm).transpose(-1, -2), fb).transpose(-1, -2)
    for name, S in (("spec", mag), ("mel", mel)):
        v = torch.log10(S) - 1
        st[f"stft/{name}"] = torch.clamp((v + 5) / 5, 0.0, 1.0).numpy()
    st["stft/audio"], st["stft/fb"], st["stft/window"] = audio, fb.numpy(), w.numpy()
    st["stft/window_mel"] = wm.numpy()
    np.savez_compressed(os.path.join(out_dir, "stft.npz"), **st)


def gen_q(torch, GaussianDiffusion, out_dir):
    """9. Forward-process noising q_stochastic / q_stochastic_conditional (diffusion.py:225-279):
    torch.manual_seed(s) before each call fixes the reference's randint / rand draws (CPU
    generator), which the tests re-draw with the same seed and hand to the library."""
    q = {}
    rng = np.random.default_rng(21)
    for sched in (("linear", 50, 1e-6, 1e-3), ("linear", 200, 1e-4, 0.02)):
        d = GaussianDiffusion(*sched, device="cpu")
        B, N = 4, 700
        x0 = rng.uniform(-0.5, 0.5, (B, 1, N)).astype(np.float32)
        y = (x0 + rng.uniform(-0.2, 0.2, (B, 1, N))).astype(np.float32)
        noise = rng.standard_normal((B, 1, N)).astype(np.float32)
        k = f"q/{sched_key(sched)}"
        q[k + "/x0"], q[k + "/y"], q[k + "/noise"] = x0, y, noise
        with torch.no_grad():
            for ti, name in ((False, "float"), (True, "int")):
                torch.manual_seed(5)
                xt, s, lvl = d.q_stochastic(torch.from_numpy(x0), torch.from_numpy(noise), t_is_integer=ti)
                q[f"{k}/{name}/x_t"], q[f"{k}/{name}/s"], q[f"{k}/{name}/level"] = xt.numpy(), s.numpy(), lvl.numpy()
            torch.manual_seed(6)
            xt, comb, s = d.q_stochastic_conditional(torch.from_numpy(x0), torch.from_numpy(y), torch.from_numpy(noise))
            q[f"{k}/cond/x_t"], q[f"{k}/cond/combined"], q[f"{k}/cond/s"] = xt.numpy(), comb.numpy(), s.numpy()
    np.savez_compressed(os.path.join(out_dir, "q_sample.npz"), **q)


def gen_wavegrad(torch, philox, make_params, GaussianDiffusion, out_dir):
    """8. WaveGrad (model/wavegrad.py) forward, and the reverse loop of SDDM_spectrogram.infer
    (model.py:212-257) with the SURVEY Q4 adapter (x_t [B,1,N] -> audio [B,N], noise level [B],
    eps reshaped to [B,1,N]): the reference wiring itself fails on WaveGrad's 4-D Conv1d input."""
    from model.wavegrad import WaveGrad
    wg = {}
    rng = np.random.default_rng(9)
    F, B = 6, 2
    net = WaveGrad()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    P = make_params(shapes, 0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    net.eval()
    spec = rng.uniform(0, 1, (B, 128, F)).astype(np.float32)
    N = 300 * F
    audio = philox.normal(17, 0, (B, N))
    nl = np.array([0.7, 0.3], dtype=np.float32)
    with torch.no_grad():
        y = net(torch.from_numpy(spec), torch.from_numpy(audio), torch.from_numpy(nl))
    key = f"wg/fw/{F}x{B}"
    wg[key + "/spec"], wg[key + "/audio"], wg[key + "/noise_level"] = spec, audio, nl
    wg[key + "/eps"] = y.numpy().copy()
    sched = ("linear", 3, 1e-4, 0.05)
    d = GaussianDiffusion(*sched, device="cpu")
    inj = NoiseInjector(torch, philox, 7)
    inj.draws = [0] + list(range(sched[1], 1, -1))
    steps = []
    with inj, torch.no_grad():
        x = torch.randn(B, 1, N)                                   # model.py:216
        for t in reversed(range(1, sched[1] + 1)):
            noise_level = d.get_noise_level(t) * torch.ones(B)     # model.py:227-229 (adapter: [B])
            eps = net(torch.from_numpy(spec), x[:, 0, :], noise_level).reshape(B, 1, N)
            x = d.p_transition(x, t, eps)
            steps.append(x.numpy().copy())
    key = f"wg/inf/sqrt_alpha_bar/{sched_key(sched)}/{F}x{B}"
    wg[key + "/spec"] = spec
    wg[key + "/out"] = x.numpy().copy()
    wg[key + "/steps"] = np.stack(steps)
    np.savez_compressed(os.path.join(out_dir, "wavegrad.npz"), **wg)
    with open(os.path.join(out_dir, "state_dict_keys.json")) as f:
        keys = json.load(f)
    keys["wavegrad"] = [[k, list(v.shape)] for k, v in net.state_dict().items()]
    with open(os.path.join(out_dir, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)


def gen_torchnoise(torch, make_params, GaussianDiffusion, noisy_speech, out_dir):
    """12. sampling loops with the reference's OWN noise (torch_noise.npz): no injection, torch seeded
    with torch.manual_seed(seed) right before infer, so every draw is the reference's torch.randn_like /
    torch.randn on the CPU generator (model.py:57-68,216; diffusion.py:172,187,207,220,285,306).
    The HIP side replays the same draws through sddm_sample_noise (SURVEY §8(b) noise_mode 1)."""
    from model.UNetModified2 import UNetModified2
    from model.model import SDDM, SDDM_spectrogram
    from model.diffwave import DiffWave
    from model.wavegrad import WaveGrad
    tn = {}
    sched, N, B = ("linear", 6, 1e-4, 0.05), 2112, 2
    net = UNetModified2(num_samples=N, **UNET_ARGS)
    P = make_params({k: tuple(v.shape) for k, v in net.state_dict().items()}, 0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    cond = noisy_speech(B, N, seed=4321)
    for i, mode in enumerate(("condition_in", "original", "sr3", "supportive", "conditional")):
        d = GaussianDiffusion(*sched, device="cpu")
        m = SDDM(d, net, p_transition=mode).eval()
        seed = 100 + i
        torch.manual_seed(seed)
        with torch.no_grad():
            y = m.infer(torch.from_numpy(cond))
        key = f"torchnoise/unet/{mode}/{sched_key(sched)}/{N}x{B}"
        tn[key + "/cond"], tn[key + "/out"], tn[key + "/seed"] = cond, y.numpy().copy(), np.array(seed)
    sched, F = ("linear", 6, 1e-4, 0.02), 16
    net = DiffWave(num_samples=-1, num_timesteps=sched[1], freq_bins=513, residual_channels=64, residual_layers=30,
                   dilation_cycle_length=10)
    P = make_params({k: tuple(v.shape) for k, v in net.state_dict().items()}, 0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    m = SDDM_spectrogram(GaussianDiffusion(*sched, device="cpu"), net, hop_samples=256,
                         noise_condition="time_step").eval()
    spec = np.random.default_rng(5).uniform(0, 1, (1, 513, F)).astype(np.float32)
    torch.manual_seed(200)
    with torch.no_grad():
        y = m.infer(torch.from_numpy(spec))
    key = f"torchnoise/diffwave/time_step/{sched_key(sched)}/{F}x1"
    tn[key + "/spec"], tn[key + "/out"], tn[key + "/seed"] = spec, y.numpy().copy(), np.array(200)
    np.savez_compressed(os.path.join(out_dir, "torch_noise.npz"), **tn)
    print("wrote", os.path.join(out_dir, "torch_noise.npz"))


def gen_long(torch, philox, make_params, GaussianDiffusion, noisy_speech, out_dir):
    """11. the long sampling loops the benches run, from the reference (long_loops.npz):
    UNet condition_in at T=1000 (config_unet.json's linear 1e-6..1e-3 at the headline's T; N=2112,
    B=2), DiffWave at T=200 (config_diffwave.json schedule and time_step condition; 63 frames, B=1)
    and WaveGrad at T=50 (SURVEY §8d fast schedule linear 1e-4..0.05; 54 frames, B=2: the reference
    WaveGrad cannot run B=1).  x_t is kept every `rec` steps to localise a divergence."""
    from model.UNetModified2 import UNetModified2
    from model.model import SDDM, SDDM_spectrogram
    from model.diffwave import DiffWave
    from model.wavegrad import WaveGrad
    lg = {}

    def recorder(d, every, T):
        steps, orig = [], d.p_transition

        def rec(x, t, *a, **kw):
            y = orig(x, t, *a, **kw)
            if t % every == 1 or every == 1:     # x_{t-1} after step t = k*every + 1: x_{k*every}
                steps.append(y.numpy().copy())
            return y
        d.p_transition = rec
        return steps

    # UNet, T = 1000
    sched, N, B = ("linear", 1000, 1e-6, 1e-3), 2112, 2
    d = GaussianDiffusion(*sched, device="cpu")
    net = UNetModified2(num_samples=N, **UNET_ARGS)
    P = make_params({k: tuple(v.shape) for k, v in net.state_dict().items()}, 0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    m = SDDM(d, net, p_transition="condition_in").eval()
    cond = noisy_speech(B, N, seed=1234)
    steps = recorder(d, 100, sched[1])
    inj = NoiseInjector(torch, philox, 7)
    inj.draws = [0] + list(range(sched[1], 1, -1))
    with inj, torch.no_grad():
        y = m.infer(torch.from_numpy(cond))
    key = f"long/unet/condition_in/{sched_key(sched)}/{N}x{B}"
    lg[key + "/cond"], lg[key + "/out"], lg[key + "/every100"] = cond, y.numpy().copy(), np.stack(steps)
    print("unet T=1000 done", flush=True)

    # DiffWave, T = 200 (config_diffwave.json), 63 frames
    sched, F, B = ("linear", 200, 1e-4, 0.02), 63, 1
    net = DiffWave(num_samples=-1, num_timesteps=sched[1], freq_bins=513, residual_channels=64,
                   residual_layers=30, dilation_cycle_length=10)
    P = make_params({k: tuple(v.shape) for k, v in net.state_dict().items()}, 0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    net.eval()
    spec = np.random.default_rng(21).uniform(0, 1, (B, 513, F)).astype(np.float32)
    d = GaussianDiffusion(*sched, device="cpu")
    m = SDDM_spectrogram(d, net, hop_samples=256, noise_condition="time_step").eval()
    steps = recorder(d, 20, sched[1])
    inj = NoiseInjector(torch, philox, 7)
    inj.draws = [0] + list(range(sched[1], 1, -1))
    with inj, torch.no_grad():
        y = m.infer(torch.from_numpy(spec))
    key = f"long/diffwave/time_step/{sched_key(sched)}/{F}x{B}"
    lg[key + "/spec"], lg[key + "/out"], lg[key + "/every20"] = spec, y.numpy().copy(), np.stack(steps)
    print("diffwave T=200 done", flush=True)

    # WaveGrad, T = 50, 54 frames (adapter of SURVEY Q4, as gen_wavegrad)
    sched, F, B = ("linear", 50, 1e-4, 0.05), 54, 2
    net = WaveGrad()
    P = make_params({k: tuple(v.shape) for k, v in net.state_dict().items()}, 0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    net.eval()
    spec = np.random.default_rng(22).uniform(0, 1, (B, 128, F)).astype(np.float32)
    N = 300 * F
    d = GaussianDiffusion(*sched, device="cpu")
    inj = NoiseInjector(torch, philox, 7)
    inj.draws = [0] + list(range(sched[1], 1, -1))
    steps = []
    with inj, torch.no_grad():
        x = torch.randn(B, 1, N)                                   # model.py:216
        for t in reversed(range(1, sched[1] + 1)):
            noise_level = d.get_noise_level(t) * torch.ones(B)     # model.py:227-229 (adapter: [B])
            eps = net(torch.from_numpy(spec), x[:, 0, :], noise_level).reshape(B, 1, N)
            x = d.p_transition(x, t, eps)
            if t % 10 == 1:
                steps.append(x.numpy().copy())
    key = f"long/wavegrad/sqrt_alpha_bar/{sched_key(sched)}/{F}x{B}"
    lg[key + "/spec"], lg[key + "/out"], lg[key + "/every10"] = spec, x.numpy().copy(), np.stack(steps)
    np.savez_compressed(os.path.join(out_dir, "long_loops.npz"), **lg)
    print("wrote", os.path.join(out_dir, "long_loops.npz"))


if __name__ == "__main__":
    main()
