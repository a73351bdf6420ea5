"""Node-local job launcher (replaces Vertex AI Training's worker pools).

CLI::

    python -m mipipe.launch --replica-count 4 --accelerator-count 2 -- \
        python -m mipipe.train.task --dist-url=env:// --multiprocessing-distributed
    python -m mipipe.launch --nproc-per-node 8 --accelerator-count 8 -- python bench.py
"""
from .launcher import LaunchSpec, ReplicaResult, build_envs, free_port, launch, visible_gpu_ids  # noqa: F401
