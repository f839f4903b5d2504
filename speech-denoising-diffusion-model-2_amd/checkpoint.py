"""Checkpoint reader for the reference's ``torch.save`` format (base/base_trainer.py:108-128;
read at infer.py:46-51): {'arch', 'epoch', 'state_dict', 'optimizer', 'monitor_best', 'config'}.

The file is loaded with ``torch.load(weights_only=True)`` only.  The non-tensor objects the
reference pickles beside the weights (its ``ConfigParser`` with ``pathlib`` paths) are not on
torch's allowlist; their class names are read from the pickle without executing it
(``get_unsafe_globals_in_checkpoint``) and each is mapped to an inert placeholder that only
records its constructor arguments and state, so nothing from the file runs.
"""
import torch


def _placeholder(qualname):
    class Opaque:
        __slots__ = ("args", "state")

        def __new__(cls, *args, **kwargs):
            o = object.__new__(cls)
            o.args, o.state = args, None
            return o

        def __init__(self, *args, **kwargs):
            pass

        def __setstate__(self, state):
            self.state = state

        def __repr__(self):
            return f"<opaque {qualname}>"

    Opaque.__name__ = Opaque.__qualname__ = qualname.rsplit(".", 1)[-1]
    return Opaque


def load_checkpoint(path, map_location="cpu"):
    names = torch.serialization.get_unsafe_globals_in_checkpoint(path)
    with torch.serialization.safe_globals([(_placeholder(n), n) for n in names]):
        return torch.load(path, map_location=map_location, weights_only=True)


def state_dict_from_checkpoint(path, map_location="cpu"):
    """The model state_dict of a reference checkpoint, with the ``module.`` prefix a
    DataParallel-trained model adds (infer.py:49-51) removed."""
    ck = load_checkpoint(path, map_location)
    sd = ck["state_dict"] if isinstance(ck, dict) and "state_dict" in ck else ck
    return {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
