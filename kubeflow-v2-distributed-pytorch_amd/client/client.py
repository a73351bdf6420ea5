"""Submission client (replaces ``kfp.v2.google.client.AIPlatformClient``).

Reference: ``AIPlatformClient(project_id=PROJECT_ID, region=REGION)`` (nb:253-258) and
``create_run_from_job_spec("dag-<ts>.json", pipeline_root=PIPELINE_ROOT,
parameter_values={"baseline_accuracy": 80.0})`` (nb:281-285), which returned a console
link with run id ``download-file<uuid>-20210824170532`` (nb:270).  Here the run executes
on the local orchestrator (:mod:`mipipe.orchestrator`); ``create_run_from_job_spec``
starts it and returns a response dict immediately (Vertex semantics), the run record is
persisted under ``<pipeline_root>/<run_id>/run.json`` and ``wait_for_run`` /
``get_run`` read it back.  ``sync=True`` blocks until the run ends.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Any, Dict, Optional

from mipipe.orchestrator.runner import PipelineRunner, TERMINAL_STATES
from mipipe.storage.gcs import uri_to_local_path

__all__ = ["AIPlatformClient", "Client", "RunHandle"]


class RunHandle:
    def __init__(self, runner: PipelineRunner, thread: Optional[threading.Thread]):
        self.runner = runner
        self.thread = thread
        self.result: Optional[Dict[str, Any]] = None
        self.error: Optional[BaseException] = None

    @property
    def run_id(self) -> str:
        return self.runner.run_id

    def wait(self, timeout: Optional[float] = None) -> Dict[str, Any]:
        if self.thread is not None:
            self.thread.join(timeout)
            if self.thread.is_alive():
                raise TimeoutError(f"run {self.run_id} still running")
        if self.error is not None:
            raise self.error
        return self.result

    @property
    def state(self) -> str:
        return self.runner.state


class AIPlatformClient:
    """Drop-in for the deprecated ``AIPlatformClient`` used by the reference notebook."""

    def __init__(self, project_id: str = "local", region: str = "local",
                 max_parallel: int = 4, echo_logs: bool = True):
        self.project_id = project_id
        self.region = region
        self.max_parallel = max_parallel
        self.echo_logs = echo_logs
        self._runs: Dict[str, RunHandle] = {}

    def create_run_from_job_spec(self, job_spec_path: str, job_id: Optional[str] = None,
                                 pipeline_root: Optional[str] = None,
                                 parameter_values: Optional[Dict[str, Any]] = None,
                                 enable_caching: Optional[bool] = None,
                                 labels: Optional[Dict[str, str]] = None,
                                 service_account: Optional[str] = None,
                                 network: Optional[str] = None,
                                 sync: bool = False) -> Dict[str, Any]:
        with open(job_spec_path) as f:
            spec = json.load(f)
        runner = PipelineRunner(spec, pipeline_root=pipeline_root,
                                parameter_values=parameter_values, run_id=job_id,
                                enable_caching=enable_caching, max_parallel=self.max_parallel,
                                echo_logs=self.echo_logs)
        handle = RunHandle(runner, None)

        def target():
            try:
                handle.result = runner.run()
            except BaseException as e:  # surfaced by wait()
                handle.error = e

        if sync:
            target()
        else:
            th = threading.Thread(target=target, name=f"mipipe-run-{runner.run_id}")
            handle.thread = th
            th.start()
        self._runs[runner.run_id] = handle
        name = f"projects/{self.project_id}/locations/{self.region}/pipelineJobs/{runner.run_id}"
        print(f"See the Pipeline job here: file://{runner.run_dir}/run.json")
        return {"name": name, "runId": runner.run_id, "displayName": runner.pipeline_name,
                "state": runner.state, "pipelineRoot": runner.pipeline_root,
                "runDir": runner.run_dir, "labels": dict(labels or {})}

    def wait_for_run(self, run_id: str, timeout: Optional[float] = None) -> Dict[str, Any]:
        if run_id in self._runs:
            return self._runs[run_id].wait(timeout)
        t0 = time.time()
        while True:
            r = self.get_run(run_id)
            if r and r["state"] in ("PIPELINE_STATE_SUCCEEDED", "PIPELINE_STATE_FAILED"):
                return r
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError(run_id)
            time.sleep(0.5)

    def get_run(self, run_id: str, pipeline_root: Optional[str] = None) -> Optional[Dict[str, Any]]:
        if run_id in self._runs:
            root = self._runs[run_id].runner.run_dir
        else:
            root = uri_to_local_path(f"{(pipeline_root or '').rstrip('/')}/{run_id}")
        p = os.path.join(root, "run.json")
        if not os.path.isfile(p):
            return None
        with open(p) as f:
            return json.load(f)

    # kfp 1.8 also exposes schedules; a local cron is out of scope — fail loudly.
    def create_schedule_from_job_spec(self, *a, **k):
        raise NotImplementedError("recurring schedules are not supported by the local orchestrator")


class Client(AIPlatformClient):
    """kfp-2-style convenience: compile + run a pipeline function in one call."""

    def create_run_from_pipeline_func(self, pipeline_func, arguments: Optional[Dict[str, Any]] = None,
                                      pipeline_root: Optional[str] = None,
                                      enable_caching: Optional[bool] = None,
                                      run_name: Optional[str] = None, sync: bool = True,
                                      package_path: Optional[str] = None) -> Dict[str, Any]:
        import tempfile
        from mipipe.compiler import Compiler
        path = package_path or os.path.join(tempfile.mkdtemp(prefix="mipipe-"), "pipeline.json")
        Compiler().compile(pipeline_func, path)
        return self.create_run_from_job_spec(path, job_id=run_name, pipeline_root=pipeline_root,
                                             parameter_values=arguments,
                                             enable_caching=enable_caching, sync=sync)
