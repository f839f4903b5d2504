"""ORACLE — CPU restatement of the reference's reverse-diffusion sampling path.

THIS PACKAGE IS TEST INFRASTRUCTURE ONLY.  It is the checker, never the thing
measured or shipped: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  The product path
(``speech-denoising-diffusion-model-2_amd/``) never imports anything from here
and fails loudly when its HIP library is missing.

Every function cites the reference file:line (paths relative to the upstream
repository yangye1098/Speech-Denoising-Diffusion-Model-2) that it restates.

Parity pinning: the reference ships no tests, fixtures or golden vectors
(SURVEY.md §4).  The oracle is pinned against golden vectors produced by
importing the reference Python in the build container with the counter-based
noise stream of ``oracle.philox`` injected in place of ``torch.randn*``
(``tests/golden/gen_golden.py``; fixtures in ``tests/golden/*.npz``).

Modules
  philox    Philox4x32-10 + Box–Muller normal stream keyed by (seed, draw, element)
  schedule  GaussianDiffusion tables (model/diffusion.py:49-161)
  transition  p_transition* / get_x_T* (model/diffusion.py:164-223, 281-320)
  unet      UNetModified2 forward (model/UNetModified2.py)
  sampler   SDDM.infer loop (model/model.py:50-124)
"""
