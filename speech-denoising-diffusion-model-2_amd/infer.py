"""Inference driver (reference infer.py:20-146): chunk every file of ``infer_dataset`` into
``num_samples``-sample pieces, denoise them with ``model.infer`` on the HIP device, stitch each
file's chunks back together and write output / target / condition WAVs under
``<save_dir>/samples``.

    python infer.py -c config.json -r checkpoint.pth [--seed S]

Differences from the reference:
  Q1  ``infer_data_loader`` defaults to {InferDataLoader, batch_size 4, num_workers 2} when the
      config lacks it (config_unet.json does);
  Q2  the last file of every batch is written too (the reference flushes a file only when the
      next index appears, so it drops one file per batch);
  Q3  no DataParallel wrapper (it cannot call ``.infer``); multi-GPU runs shard rows instead:
      under ``torchrun --nproc-per-node P infer.py ...`` every rank samples a contiguous block of
      each batch's rows (model.sharded_infer: row_offset-keyed noise, one RCCL all-gather), so the
      written files equal a single-GPU run bit for bit; rank 0 writes them;
  the PESQ/STOI evaluation step needs torchmetrics (absent): the loss and SI-SNR are logged.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import data_loader.data_loaders as module_data  # noqa: E402
import model.diffusion as module_diffusion  # noqa: E402
import model.loss as module_loss  # noqa: E402
import model.metric as module_metric  # noqa: E402
import model.model as module_arch  # noqa: E402
import model.network as module_network  # noqa: E402
from checkpoint import state_dict_from_checkpoint  # noqa: E402
from data_loader import wav_io  # noqa: E402
from parse_config import ConfigParser  # noqa: E402

EXPAND_ORDER = 3


def log_modulus_normalize_reverse(audio_log_modulus, expand_order):
    """prepare_logaudio.py:22-26."""
    audio_log_modulus = audio_log_modulus * 2 * expand_order
    sign = torch.sign(audio_log_modulus)
    return sign * (torch.pow(10, torch.abs(audio_log_modulus)) - 1.) / 10. ** expand_order


def regroup(index):
    """Runs of equal file index in a collated batch -> [(file index, [rows])] (infer.py:81-120,
    with the final run flushed: SURVEY Q2)."""
    groups = []
    for b, ind in enumerate(index.tolist()):
        if groups and groups[-1][0] == ind:
            groups[-1][1].append(b)
        else:
            groups.append((ind, [b]))
    return groups


def write_file(paths, name, output, target, condition, rows, datatype, sample_rate):
    for tensor, path in ((output, paths["output"]), (target, paths["target"]), (condition, paths["condition"])):
        one = tensor[rows, :, :].reshape(1, -1).float().cpu()
        if datatype == ".logwav.npy":
            one = log_modulus_normalize_reverse(one, EXPAND_ORDER)
        wav_io.save(os.path.join(path, f"{name}.wav"), one, sample_rate)


def run(config, model, loader, dataset, device, logger=None, seed=None):
    """The loop of infer.py:70-128; returns the mean loss and SI-SNR over batches."""
    import torch.distributed as dist
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    datatype = dataset.datatype
    sample_rate = config["sample_rate"]
    sample_path = os.path.join(str(config.save_dir), "samples")
    paths = {k: os.path.join(sample_path, k) for k in ("target", "output", "condition")}
    for p in paths.values():
        os.makedirs(p, exist_ok=True)
    loss_fn = getattr(module_loss, config["loss"]) if "loss" in config.config else module_loss.l1_loss
    total_loss, total_sisnr, n = 0.0, 0.0, 0
    with torch.no_grad():
        for i, (target, condition, index) in enumerate(loader):
            target, condition = target.to(device), condition.to(device)
            output = module_arch.sharded_infer(model, condition, seed=None if seed is None else seed + i)
            if rank != 0:
                continue
            for ind, rows in regroup(index):
                write_file(paths, dataset.getName(ind), output, target, condition, rows, datatype, sample_rate)
            total_loss += float(loss_fn(output, target))
            total_sisnr += float(module_metric.sisnr(output, target))
            n += 1
    log = {"loss": total_loss / max(n, 1), "sisnr": total_sisnr / max(n, 1)}
    if logger and rank == 0:
        logger.info(log)
    return log


def main(config, seed=None, lane_rows=None):
    logger = config.get_logger("infer")
    if "infer_data_loader" not in config.config:
        config.config["infer_data_loader"] = {"type": "InferDataLoader", "args": {"batch_size": 4, "num_workers": 2}}
    infer_dataset = config.init_obj("infer_dataset", module_data, sample_rate=config["sample_rate"],
                                    T=config["num_samples"])
    infer_data_loader = config.init_obj("infer_data_loader", module_data, infer_dataset)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:                                   # torchrun: one process per GPU, RCCL over xGMI
        import torch.distributed as dist
        # bind the rank's device before the process group, and hand it to RCCL (its communicator
        # lives on that device)
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    device = torch.device("cuda", torch.cuda.current_device())
    _, _, model = module_arch.build_from_config(config, module_diffusion, module_network, module_arch, device)
    model = model.to(device).eval()
    # rows per lane of the UNet plan (library default 16): small batches (a few chunks of
    # InferDataLoader's 4 files) run faster on lane_rows 4 / 8 plans, which have their own measured
    # kernel tables in configs/conv_tuning.json.  --lane-rows or a top-level "lane_rows" config key.
    lane_rows = lane_rows or config.config.get("lane_rows")
    if lane_rows:
        model.lane_rows = int(lane_rows)
    if config.resume is not None:
        logger.info("Loading checkpoint: {} ...".format(config.resume))
        model.load_state_dict(state_dict_from_checkpoint(str(config.resume)))
    return run(config, model, infer_data_loader, infer_dataset, device, logger, seed)


if __name__ == "__main__":
    args = argparse.ArgumentParser(description="SDDM inference on MI355X")
    args.add_argument("-c", "--config", default=None, type=str, help="config file path")
    args.add_argument("-r", "--resume", default=None, type=str, help="checkpoint path")
    args.add_argument("-d", "--device", default=None, type=str, help="indices of GPUs to enable")
    args.add_argument("--seed", default=None, type=int, help="noise seed (default: torch's generator)")
    args.add_argument("--lane-rows", default=None, type=int, help="rows per UNet lane (default: the library's 16)")
    seed, lane = None, None
    if "--seed" in sys.argv:
        k = sys.argv.index("--seed")
        seed = int(sys.argv[k + 1])
        del sys.argv[k:k + 2]
    if "--lane-rows" in sys.argv:
        k = sys.argv.index("--lane-rows")
        lane = int(sys.argv[k + 1])
        del sys.argv[k:k + 2]
    main(ConfigParser.from_args(args), seed, lane)
