"""Distributed training entry point — flag-compatible with the reference's ``task.py``.

Reference: /root/reference/task.py (318 lines).  Same CLI flags with the same names and
defaults (task.py:55-95) so the compiled pipeline's args
(``--dist-url=env:// --multiprocessing-distributed --num_epochs=2``, nb:159-163) work
unchanged, the same env contract (``WORLD_SIZE``/``RANK``/``MASTER_*``/``AIP_MODEL_DIR``) and
the same process structure: ``main()`` resolves the distributed mode (task.py:97-113) and
either ``mp.spawn``s one worker per local GPU (task.py:117-124) or runs ``main_worker``
in-process (task.py:127); ``main_worker`` does rank math + rendezvous (task.py:132-150),
seeding (161-162), model construction (165-171), DDP wrapping (173-208), loss/optimizer
(210-214), resume (216-242), data (246-267), the epoch loop with periodic eval + export
(272-312).

Deliberate fixes of reference quirks, each noted inline:
  * evaluation runs on the *unwrapped* model, sharded over all ranks (no rank-0-only
    collective mismatch, §5.2); the model is also evaluated and saved after training;
  * ``--resume`` takes a path (or ``auto``) and ``start_epoch`` is honoured;
  * ``DistributedSampler.set_epoch`` is called; ``--dist-url`` defaults to ``env://``;
  * per-process batch = ``--batch_size`` (what the reference effectively does), reported
    together with the global batch;
  * data is synthetic and generated on the GPU (no download race, no CPU decode).
Additions: ``--dtype``, ``--dataset``, ``--steps``, ``--bench``, ``--num_classes``,
``--eval-every``, metrics JSON with samples/sec, fault injection for tests.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time
from datetime import datetime

if __package__ in (None, ""):  # executed as a plain script (the pipeline stages it as task.py)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch
import torch.multiprocessing as mp

from mipipe.models import create_model, model_names
from mipipe.obs import trace
from mipipe.obs.log import JsonlLogger
from mipipe.launch.env import device_offset, local_gpus
from mipipe.parallel import DataParallel, DistributedDataParallel, DistributedSampler
from mipipe.parallel import dist_utils
from mipipe.data.synthetic import DATASET_SHAPES, DeviceBatchLoader, SyntheticImageDataset
from mipipe.optim import SGD
from mipipe.ops import functional as MF
from mipipe.train import checkpoint as ckpt
from mipipe.obs.meter import ThroughputMeter

best_acc1 = 0.0


def set_random_seeds(random_seed: int = 0) -> None:
    """task.py:22-28: seed torch / numpy / random.  The reference's
    ``cudnn.deterministic = True`` maps to mipipe's deterministic mode (``--deterministic``,
    see :func:`configure_kernels`)."""
    torch.manual_seed(random_seed)
    np.random.seed(random_seed)
    random.seed(random_seed)


def configure_kernels(use_gpu: bool, deterministic: bool = True) -> None:
    """task.py:25-26 ``cudnn.deterministic = True`` -> mipipe's deterministic mode (fixed-order
    reductions, no float atomics: :mod:`mipipe.ops.determinism`); task.py:244
    ``cudnn.benchmark = True`` -> per-shape tile autotuning of the conv kernels
    (:mod:`mipipe.ops.tuning`; ``MIPIPE_BENCHMARK=0`` disables it, ``MIPIPE_TUNE_TABLE=path``
    starts from a saved table).  In deterministic mode nothing is picked by timing (the plan
    fixes the reduction order): a loaded / shipped table or the heuristic decides."""
    if not use_gpu:
        return
    from mipipe.ops import determinism, tuning
    determinism.set_deterministic(deterministic)
    tuning.from_env(deterministic)  # deterministic: shipped measured tables replace timing
    tuning.set_benchmark(os.environ.get("MIPIPE_BENCHMARK", "1") != "0",
                         verbose=os.environ.get("MIPIPE_TUNE_VERBOSE", "0") == "1")


class CrossEntropyLoss(torch.nn.Module):
    """``nn.CrossEntropyLoss()`` (task.py:211) on the fused log-softmax+NLL kernel."""

    def __init__(self, label_smoothing: float = 0.0, ignore_index: int = -100):
        super().__init__()
        self.label_smoothing = label_smoothing
        self.ignore_index = ignore_index

    def _ce(self, logits, labels):
        return MF.cross_entropy(logits, labels, self.label_smoothing, self.ignore_index)

    def forward(self, logits, labels):
        if isinstance(logits, tuple) and hasattr(logits, "_fields"):
            # GoogLeNet / Inception-v3 in training mode return torchvision's named tuples
            # (main logits + auxiliary classifiers).  The reference hands them to
            # nn.CrossEntropyLoss (task.py:310) and crashes; here the auxiliary losses are added
            # with the papers' weights: 0.3 per GoogLeNet head, 0.4 for Inception-v3's.
            w = 0.4 if len(logits) == 2 else 0.3
            loss = self._ce(logits[0], labels)
            for aux in logits[1:]:
                if aux is not None:
                    loss = loss + w * self._ce(aux, labels)
            return loss
        return self._ce(logits, labels)


def _unwrap(model):
    return model.module if isinstance(model, (DistributedDataParallel, DataParallel,
                                          torch.nn.DataParallel)) else model


@torch.no_grad()
def evaluate(model, device, test_loader) -> float:
    """Top-1 accuracy (task.py:30-46) — argmax + correct count run in ONE fused kernel per
    batch (``top1_correct``, accumulating into a device counter) and the host reads one value
    at the end instead of a ``.item()`` per batch.  Sharded over ranks (each rank's loader
    holds its shard) and summed with one all-reduce."""
    from mipipe.ops import kernels as K
    m = _unwrap(model)
    was_training = m.training
    m.eval()
    correct = torch.zeros(1, dtype=torch.int32, device=device)
    total = 0
    for images, labels in test_loader:
        images, labels = images.to(device), labels.to(device)
        outputs = m(images)
        K.top1_correct(outputs, labels, correct)
        total += labels.numel()
    t = torch.stack([correct[0].to(torch.int64), torch.tensor(total, device=device)])
    if dist_utils.get_world_size() > 1:
        torch.distributed.all_reduce(t)
    if was_training:
        m.train()
    return float(t[0].item()) / max(1, int(t[1].item()))


def build_parser() -> argparse.ArgumentParser:
    names = model_names()
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                                description="mipipe distributed trainer (task.py compatible)")
    # --- reference flags (task.py:56-94), same names and defaults -------------------------
    p.add_argument("--local_rank", type=int, help="Local rank (torch.distributed.launch compat).")
    p.add_argument("--num_epochs", type=int, default=100, help="Number of training epochs.")
    p.add_argument("--batch_size", type=int, default=1024, help="Training batch size for one process.")
    p.add_argument("--learning_rate", dest="learning_rate", type=float, default=0.1, help="Learning rate.")
    p.add_argument("--random_seed", type=int, default=0, help="Random seed.")
    p.add_argument("--model_dir", type=str, default=os.environ.get("AIP_MODEL_DIR", ""),
                   help="Directory (or gs:// URI) for saving models.")
    p.add_argument("--model_filename", type=str, default="resnet_distributed.pth", help="Model filename.")
    p.add_argument("-a", "--arch", metavar="ARCH", default="resnet18", choices=names,
                   help="model architecture: " + " | ".join(names) + " (default: resnet18)")
    p.add_argument("--momentum", default=0.9, type=float, metavar="M", help="momentum")
    p.add_argument("--wd", "--weight-decay", default=1e-4, type=float, metavar="W",
                   dest="weight_decay", help="weight decay (default: 1e-4)")
    p.add_argument("--pretrained", dest="pretrained", action="store_true",
                   help="use pre-trained model: torchvision-format weights from "
                        "--pretrained-weights or the torchvision cache (no network download)")
    p.add_argument("--pretrained-weights", dest="pretrained_weights", default=None,
                   help="path of a torchvision-format state_dict (.pth) for --pretrained")
    p.add_argument("--local_training", dest="local_training", action="store_true",
                   help="save to --model_dir instead of AIP_MODEL_DIR")
    p.add_argument("--rank", default=-1, type=int, help="node rank for distributed training")
    p.add_argument("--resume", nargs="?", const="auto", default="",
                   help="resume from checkpoint PATH ('auto' = <model_dir>/checkpoint.pth.tar)")
    p.add_argument("--world-size", default=int(os.getenv("WORLD_SIZE", -1)), type=int,
                   help="number of nodes for distributed training")
    p.add_argument("--dist-url", default="env://", type=str,
                   help="url used to set up distributed training (reference default "
                        "http://localhost:8082 is not a valid init method)")
    p.add_argument("--dist-backend", default="nccl", type=str,
                   help="distributed backend (nccl = RCCL on ROCm; gloo on CPU)")
    p.add_argument("--multiprocessing-distributed", action="store_true",
                   help="launch one process per local GPU (N per node)")
    p.add_argument("--gpu", default=None, type=int, help="GPU id to use.")
    p.add_argument("--workers", default=4, type=int, metavar="N",
                   help="data loading workers (data is generated on the device; kept for compat)")
    # --- additions ------------------------------------------------------------------------
    p.add_argument("--dataset", default="cifar10", choices=sorted(DATASET_SHAPES),
                   help="synthetic dataset shape")
    p.add_argument("--image-size", type=int, default=None, help="override image H=W")
    p.add_argument("--data-dir", default="",
                   help="directory with CIFAR-binary record files (<dataset>_{train,test}.bin or "
                        "cifar-10-batches-bin/); read by the native loader. Empty: synthetic "
                        "on-device data")
    p.add_argument("--train-samples", type=int, default=None)
    p.add_argument("--test-samples", type=int, default=None)
    p.add_argument("--num_classes", type=int, default=None,
                   help="classifier width (reference keeps torchvision's 1000)")
    p.add_argument("--deterministic", dest="deterministic", action="store_true", default=True,
                   help="fixed-order reductions, bit-reproducible runs (reference task.py:25-26 "
                        "sets cudnn.deterministic); default on")
    p.add_argument("--no-deterministic", dest="deterministic", action="store_false",
                   help="allow float-atomic reductions (faster)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                   help="compute dtype on GPU (master weights stay fp32); CPU runs fp32")
    p.add_argument("--hip-graph", action="store_true",
                   help="replay full-size training steps (forward, backward with the DDP bucket "
                        "all-reduces, SGD) from one captured hipGraph; partial batches run eagerly")
    p.add_argument("--steps", type=int, default=0, help="max training steps per epoch (0 = all)")
    p.add_argument("--eval-every", type=int, default=10, help="evaluate every N epochs (task.py:279)")
    p.add_argument("--log-every", type=int, default=20)
    p.add_argument("--warmup-steps", type=int, default=2, help="steps excluded from samples/sec")
    p.add_argument("--bucket-cap-mb", type=float, default=32.0)
    p.add_argument("--no-broadcast-buffers", action="store_true")
    p.add_argument("--dist-timeout", type=float, default=1800.0, help="collective timeout (s)")
    p.add_argument("--compat-nested-model-dir", action="store_true",
                   help="export to AIP_MODEL_DIR/model/<file> like task.py:291")
    p.add_argument("--metrics-file", default="", help="write final metrics JSON here")
    p.add_argument("--trace", action="store_true",
                   help="roctx ranges around step phases (for rocprofv3 --marker-trace)")
    p.add_argument("--log-dir", default=os.environ.get("MIPIPE_LOG_DIR", ""),
                   help="per-rank JSON-lines logs (rank<k>.jsonl)")
    p.add_argument("--cpu-procs", type=int, default=1,
                   help="processes per node when no GPU is visible (gloo)")
    return p


def _ngpus() -> int:
    """GPUs of this node (replica): the launcher's MIPIPE_LOCAL_GPUS when it set one
    (launch/env.py), else every visible device."""
    if os.environ.get("MIPIPE_FORCE_CPU") == "1":
        return 0
    n = local_gpus()
    return n if n is not None else torch.cuda.device_count()


def main(argv=None) -> int:
    argv = build_parser().parse_args(argv)
    if argv.dist_url == "env://" and argv.world_size == -1:
        argv.world_size = int(os.environ.get("WORLD_SIZE", 1))
    argv.distributed = argv.world_size > 1 or argv.multiprocessing_distributed
    ngpus_per_node = _ngpus()
    procs_per_node = ngpus_per_node if ngpus_per_node > 0 else argv.cpu_procs
    if ngpus_per_node == 0:
        argv.dist_backend = "gloo"
    # debugging (task.py:104-113)
    print(f"os WORLD_SIZE={os.getenv('WORLD_SIZE', -1)}")
    print(f"os RANK={os.getenv('RANK', 0)}")
    print(f"os MASTER_ADDR={os.getenv('MASTER_ADDR', 'localhost')}")
    print(f"os MASTER_PORT={os.getenv('MASTER_PORT', '8082')}")
    print(f"Arg - distributed={argv.distributed}")
    print(f"Arg - multiprocessing_distributed={argv.multiprocessing_distributed}")
    print(f"Arg - dist_backend={argv.dist_backend}")
    print(f"Arg - dist_url={argv.dist_url}")
    print(f"ngpus_per_node={ngpus_per_node}")
    start = datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
    print(f"Starting training: {start}", flush=True)
    if argv.multiprocessing_distributed:
        argv.world_size = procs_per_node * argv.world_size  # task.py:120
        print(f"GPU x WORLD SIZE = {argv.world_size}")
        mp.spawn(main_worker, nprocs=procs_per_node, args=(procs_per_node, argv))
    else:
        main_worker(argv.gpu, procs_per_node, argv)
    end = datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
    print(f"Training complete: {end}", flush=True)
    return 0


def _fault_check(rank: int, step: int) -> None:
    spec = os.environ.get("MIPIPE_FAULT_INJECT")  # "rank:step[:code]"
    if not spec:
        return
    parts = spec.split(":")
    if int(parts[0]) == rank and int(parts[1]) == step:
        code = int(parts[2]) if len(parts) > 2 else 17
        print(f"[fault-injection] rank {rank} exiting with {code} at step {step}", flush=True)
        sys.stdout.flush()
        os._exit(code)


def main_worker(gpu, ngpus_per_node, args) -> dict:
    global best_acc1
    args.gpu = gpu
    if args.gpu is not None:
        print(f"Use GPU: {args.gpu} for training")
    if args.distributed:
        if args.dist_url == "env://" and args.rank == -1:
            args.rank = int(os.environ.get("RANK", 0))
            print(f"Distributed and getting rank from os.environ: rank={args.rank}")
        if args.multiprocessing_distributed:
            args.rank = dist_utils.global_rank(args.rank, ngpus_per_node, gpu)  # task.py:146
            print(f"Distributed and Multiprocesing. Setting rank for each worker. rank={args.rank}")
    else:
        args.rank = 0
    use_gpu = _ngpus() > 0
    if use_gpu:
        local = args.gpu if args.gpu is not None else int(os.environ.get("LOCAL_RANK", 0))
        local += device_offset()  # this replica's first GPU (launch/env.py)
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if args.distributed:
        dist_utils.init_distributed(args.dist_backend, args.dist_url, args.world_size, args.rank,
                                    args.dist_timeout, device if use_gpu else None)
        print("Process group initialized", flush=True)
    world = dist_utils.get_world_size()
    set_random_seeds(args.random_seed)  # same seed on every rank -> identical init (task.py:161)
    # cudnn.deterministic (task.py:25-26) / cudnn.benchmark (task.py:244) analogues
    configure_kernels(use_gpu, args.deterministic)

    if args.pretrained:
        print(f"=> using pre-trained model '{args.arch}'")  # task.py:167
    else:
        print(f"=> creating model '{args.arch}'")
    C, H, W, K, N = DATASET_SHAPES[args.dataset]
    if args.image_size:
        H = W = args.image_size
    kw = {}
    if args.num_classes is not None:
        kw["num_classes"] = args.num_classes
    if args.arch == "mnist_cnn":
        kw.setdefault("num_classes", K)
        kw["in_chans"] = C
    elif args.arch.startswith(("resnet", "wide_resnet", "resnext")):
        kw["in_chans"] = C
    model = create_model(args.arch, **kw)
    if args.pretrained:
        from mipipe.models import find_pretrained, load_pretrained
        wpath = find_pretrained(args.arch, args.pretrained_weights)
        if wpath is None:
            print(f"=> no local pre-trained weights for '{args.arch}' (no network access to "
                  "download them): random init")
        else:
            load_pretrained(model, wpath)
            print(f"=> loaded pre-trained weights from {wpath}")
    compute_dtype = torch.bfloat16 if (use_gpu and args.dtype == "bf16") else torch.float32
    if hasattr(model, "compute_dtype"):
        model.compute_dtype = compute_dtype
    model = model.to(device)
    if args.distributed:
        model = DistributedDataParallel(model, device_ids=[device.index] if use_gpu else None,
                                        bucket_cap_mb=args.bucket_cap_mb,
                                        broadcast_buffers=not args.no_broadcast_buffers)
    elif use_gpu and args.gpu is None and _ngpus() > 1:
        model = DataParallel(model)  # task.py:201-208 path (d), on this replica's GPUs
    criterion = CrossEntropyLoss().to(device)
    optimizer = SGD(model.parameters(), args.learning_rate, momentum=args.momentum,
                    weight_decay=args.weight_decay,
                    shadow_dtype=compute_dtype if compute_dtype != torch.float32 else None)

    start_epoch = 0
    if args.resume:
        path = ckpt.resolve_resume_path(args.resume, args.model_dir)
        if path and os.path.isfile(path):
            print(f"=> loading checkpoint '{path}'")
            state = ckpt.load_checkpoint(path, device)
            start_epoch = int(state["epoch"])
            best_acc1 = float(state.get("best_acc1", 0.0))
            ckpt.load_model_state(model, state["state_dict"])
            ckpt.restore_model_step(model, state)
            optimizer.load_state_dict(state["optimizer"])
            print(f"=> loaded checkpoint '{path}' (epoch {start_epoch})")
        else:
            print(f"=> no checkpoint found at '{path}'")

    train_files = test_files = []
    if args.data_dir:
        from mipipe.data import records as REC
        train_files = REC.dataset_files(args.data_dir, args.dataset, "train")
        test_files = REC.dataset_files(args.data_dir, args.dataset, "test")
        if not train_files:
            raise FileNotFoundError(f"no {args.dataset} record files in {args.data_dir}")
    if train_files:
        # task.py:246-267: RandomCrop(32, 4) + flip + Normalize, DistributedSampler shards,
        # test loader batch 128 unshuffled — on the native multi-threaded loader
        from mipipe.data import records as REC
        mean, std = ((REC.MNIST_MEAN, REC.MNIST_STD) if args.dataset == "mnist"
                     else (REC.CIFAR10_MEAN, REC.CIFAR10_STD))
        pad = 4 if args.dataset == "cifar10" else 0
        probe = REC.RecordDataLoader(train_files, (C, H, W), args.batch_size, train=True,
                                     pad=pad, mean=mean, std=std, seed=args.random_seed,
                                     workers=max(1, args.workers), device=device)
        train_sampler = DistributedSampler(probe.num_samples_total, seed=args.random_seed)
        probe.sampler = train_sampler
        train_loader = probe
        tfiles = test_files or train_files
        test_loader = REC.RecordDataLoader(tfiles, (C, H, W), 128, train=False, mean=mean,
                                           std=std, workers=max(1, args.workers), device=device)
        test_sampler = DistributedSampler(test_loader.num_samples_total, shuffle=False)
        test_loader.sampler = test_sampler
    else:
        train_n = args.train_samples or N
        test_n = args.test_samples or min(N, 10000)
        train_set = SyntheticImageDataset(args.dataset, train_n, seed=args.random_seed,
                                          shape=(C, H, W), num_classes=K)
        test_set = SyntheticImageDataset(args.dataset, test_n, seed=args.random_seed,
                                         shape=(C, H, W), num_classes=K)
        train_sampler = DistributedSampler(train_set, seed=args.random_seed)
        test_sampler = DistributedSampler(test_set, shuffle=False)
        train_loader = DeviceBatchLoader(train_set, args.batch_size, train_sampler, device)
        test_loader = DeviceBatchLoader(test_set, 128, test_sampler, device)

    meter = ThroughputMeter(device, warmup_steps=args.warmup_steps)
    jlog = JsonlLogger(args.rank, args.log_dir or None)
    if args.trace:
        trace.enable(True)
    global_step = 0
    last_loss = float("nan")
    accuracy = None
    # --hip-graph: the first full-size batch runs eagerly inside GraphedStep (a real training
    # step: warmup=1), which then captures the step; later batches of that shape replay it
    graphed, graph_shape = None, None
    if args.hip_graph:
        from mipipe.train.graph import GraphedStep, graph_safe
        ok, why = graph_safe(_unwrap(model), optimizer) if use_gpu else (False, "no GPU")
        if isinstance(model, DataParallel):
            ok, why = False, "DataParallel runs replicas on host threads"
        if not ok:
            print(f"=> --hip-graph off: {why}", flush=True)
            args.hip_graph = False

    def _train_step(x, y):
        optimizer.zero_grad()
        loss_ = criterion(model(x), y)
        loss_.backward()
        optimizer.step()
        return loss_

    for epoch in range(start_epoch, args.num_epochs):
        epoch_start = datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
        print(f"Rank: {args.rank}, Epoch: {epoch}, Training start: {epoch_start}", flush=True)
        train_sampler.set_epoch(epoch)
        if epoch % args.eval_every == 0:
            accuracy = evaluate(model, device, test_loader)
            if args.rank == 0:
                ckpt.export_model(model, args, epoch, accuracy)
                print("-" * 75)
                print(f"Epoch: {epoch}, Accuracy: {accuracy}, Time: "
                      f"{datetime.now().strftime('%Y_%m_%d_%H_%M_%S')}")
                print("-" * 75, flush=True)
        model.train()
        it = iter(train_loader)
        i = 0
        while True:
            if args.steps and i >= args.steps:
                break
            with trace.phase("data"):
                batch = next(it, None)
            if batch is None:
                break
            inputs, labels = batch
            _fault_check(args.rank, global_step)
            meter.step_begin()
            if args.hip_graph and (graphed is None or tuple(inputs.shape) == graph_shape):
                with trace.phase("graph_step"):
                    if graphed is None:
                        graphed = GraphedStep(_train_step, (inputs, labels), warmup=1)
                        graph_shape = tuple(inputs.shape)
                        loss = graphed.warmup_loss  # the eager warm-up step trained this batch
                    else:
                        loss = graphed.step(inputs, labels)
            else:
                with trace.phase("zero_grad"):
                    optimizer.zero_grad()
                with trace.phase("forward"):
                    outputs = model(inputs)
                    loss = criterion(outputs, labels)
                with trace.phase("backward+allreduce"):
                    loss.backward()
                with trace.phase("optimizer"):
                    optimizer.step()
            meter.step_end(inputs.shape[0])
            global_step += 1
            i += 1
            if args.log_every and global_step % args.log_every == 0:
                if isinstance(model, DistributedDataParallel):
                    model.check_comm_errors()  # a one-shot wait that gave up -> error, no sync
                last_loss = float(loss.detach().float().item())
                jlog.log("step", epoch=epoch, step=global_step, loss=last_loss,
                         samples_per_sec=meter.samples_per_sec())
                if args.rank == 0:
                    print(f"epoch {epoch} step {global_step} loss {last_loss:.4f} "
                          f"{meter.samples_per_sec() * world:.1f} samples/s (job)", flush=True)
        if args.rank == 0:
            ckpt.save_checkpoint(model, optimizer, args, epoch + 1, best_acc1)
    if isinstance(model, DistributedDataParallel):
        model.check_comm_errors(final=True)
    # fixed quirk: evaluate and save the *trained* model at the end as well
    accuracy = evaluate(model, device, test_loader)
    best_acc1 = max(best_acc1, accuracy)
    last_loss = float(loss.detach().float().item()) if global_step else last_loss
    metrics = {"accuracy": accuracy, "loss": last_loss, "epochs": args.num_epochs,
               "steps": global_step, "world_size": world, "arch": args.arch,
               "batch_per_process": args.batch_size, "global_batch": args.batch_size * world,
               "samples_per_sec_per_rank": meter.samples_per_sec(),
               "samples_per_sec_job": meter.samples_per_sec() * world,
               "dtype": str(compute_dtype).replace("torch.", ""), "device": str(device),
               "backend": (torch.distributed.get_backend() if args.distributed else "none"),
               "hip_graph": bool(args.hip_graph), "deterministic": bool(args.deterministic)}
    if args.rank == 0:
        ckpt.export_model(model, args, args.num_epochs, accuracy)
        ckpt.save_checkpoint(model, optimizer, args, args.num_epochs, best_acc1)
        print("MIPIPE_METRICS " + json.dumps(metrics), flush=True)
        if args.metrics_file:
            ckpt.write_json(args.metrics_file, metrics)
    jlog.log("final", **metrics)
    jlog.close()
    epoch_end = datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
    print(f"Epoch complete: {epoch_end}", flush=True)
    dist_utils.barrier(device if use_gpu else None)
    dist_utils.cleanup()
    return metrics


if __name__ == "__main__":
    sys.exit(main())
