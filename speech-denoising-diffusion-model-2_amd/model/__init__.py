"""Drop-in facade of the reference's ``model`` package for the sampling hot path.

Module paths and class names follow the reference (model.model.SDDM, model.diffusion.
GaussianDiffusion, model.network.UNetModified2) so ``ConfigParser.init_obj`` resolves the
reference's config.json files unchanged.  All computation goes through libsddm_hip.
"""
