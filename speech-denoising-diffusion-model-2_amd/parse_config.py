"""ConfigParser — the reference's plugin surface (parse_config.py:12-159), kept so config.json
files resolve unchanged: ``config.init_obj('network', module_network, num_samples=...)`` returns
``module_network.<type>(**args, **kwargs)``.

Run directories follow the reference (``save_dir/name/MMDD_HHMMSS`` with the config written
into it); pass ``save_dir=None`` in the trainer block to skip creating them.
"""
import json
import logging
import os
from collections import OrderedDict
from datetime import datetime
from functools import partial, reduce
from operator import getitem
from pathlib import Path


def read_json(fname):
    with Path(fname).open("rt") as f:
        return json.load(f, object_hook=OrderedDict)


def write_json(content, fname):
    with Path(fname).open("wt") as f:
        json.dump(content, f, indent=4, sort_keys=False)


def _apply_modification(config, modification):
    """Set keychain 'a;b;c' -> value entries (parse_config.py:137-159)."""
    for chain, value in (modification or {}).items():
        if value is None:
            continue
        keys = chain.split(";")
        reduce(getitem, keys[:-1], config)[keys[-1]] = value
    return config


class ConfigParser:
    def __init__(self, config, resume=None, modification=None, run_id=None):
        self._config = _apply_modification(config, modification)
        self.resume = resume
        save_root = self._config.get("trainer", {}).get("save_dir", None)
        self._save_dir = None
        if save_root is not None:
            if run_id is None:
                run_id = datetime.now().strftime(r"%m%d_%H%M%S")
            self._save_dir = Path(save_root) / self._config["name"] / run_id
            self._save_dir.mkdir(parents=True, exist_ok=(run_id == ""))
            write_json(self._config, self._save_dir / "config.json")
        self.log_levels = {0: logging.WARNING, 1: logging.INFO, 2: logging.DEBUG}

    @classmethod
    def from_args(cls, args, options=""):
        """-c/--config, -r/--resume, -d/--device CLI handling (parse_config.py:52-80)."""
        for opt in options:
            args.add_argument(*opt.flags, default=None, type=opt.type)
        if not isinstance(args, tuple) and hasattr(args, "parse_args"):
            args = args.parse_args()
        if getattr(args, "device", None) is not None:
            os.environ["HIP_VISIBLE_DEVICES"] = args.device
        if getattr(args, "resume", None) is not None:
            resume = Path(args.resume)
            cfg_fname = resume.parent / "config.json"
        else:
            assert args.config is not None, \
                "Configuration file need to be specified. Add '-c config.json', for example."
            resume = None
            cfg_fname = Path(args.config)
        config = read_json(cfg_fname)
        if args.config and resume:
            config.update(read_json(args.config))
        modification = {opt.target: getattr(args, opt.flags[-1].lstrip("-").replace("-", "_")) for opt in options}
        return cls(config, resume, modification)

    def init_obj(self, name, module, *args, **kwargs):
        """module.<config[name]['type']>(*args, **config[name]['args'], **kwargs) (parse_config.py:82-95)."""
        module_name = self[name]["type"]
        module_args = dict(self[name].get("args", {}))
        assert all(k not in module_args for k in kwargs), "Overwriting kwargs given in config file is not allowed"
        module_args.update(kwargs)
        return getattr(module, module_name)(*args, **module_args)

    def init_ftn(self, name, module, *args, **kwargs):
        module_name = self[name]["type"]
        module_args = dict(self[name].get("args", {}))
        assert all(k not in module_args for k in kwargs), "Overwriting kwargs given in config file is not allowed"
        module_args.update(kwargs)
        return partial(getattr(module, module_name), *args, **module_args)

    def __getitem__(self, name):
        return self._config[name]

    def get(self, name, default=None):
        return self._config.get(name, default)

    def get_logger(self, name, verbosity=2):
        logger = logging.getLogger(name)
        logger.setLevel(self.log_levels[verbosity])
        return logger

    @property
    def config(self):
        return self._config

    @property
    def save_dir(self):
        return self._save_dir

    @property
    def log_dir(self):
        return self._save_dir
