import argparse
import sys

from .launcher import LaunchSpec, launch


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m mipipe.launch",
                                 description="fail-fast multi-replica launcher")
    ap.add_argument("--replica-count", type=int, default=1)
    ap.add_argument("--accelerator-count", type=int, default=0, help="GPUs per replica")
    ap.add_argument("--nproc-per-node", type=int, default=None,
                    help="torchrun mode: one process per GPU of each replica")
    ap.add_argument("--model-dir", default=None, help="AIP_MODEL_DIR")
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--gpu-visibility", default="auto", choices=["auto", "slice", "all"],
                    help="slice: each replica sees only its GPUs; all: every GPU visible, "
                         "slice named by MIPIPE_DEVICE_OFFSET (launch/env.py)")
    ap.add_argument("command", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.command[1:] if a.command and a.command[0] == "--" else a.command
    if not cmd:
        ap.error("missing command")
    return launch(LaunchSpec(command=cmd, replica_count=a.replica_count,
                             accelerator_count=a.accelerator_count,
                             nproc_per_node=a.nproc_per_node, model_dir=a.model_dir,
                             log_dir=a.log_dir, master_port=a.master_port, timeout=a.timeout,
                             gpu_visibility=a.gpu_visibility))


if __name__ == "__main__":
    sys.exit(main())
