"""Local pipeline orchestrator — runs a compiled kfp v2 job spec on this node.

Replaces Vertex AI Pipelines (schedules the DAG in dependency order,
one isolated process per step, artifacts passed through ``pipeline_root``; evidence
nb:81, nb:270, pipeline.png).  Features:

* topological scheduling with independent steps running concurrently;
* sub-DAGs (``dsl.Condition`` groups) with CEL ``triggerPolicy.condition`` gates and
  ``ALL_UPSTREAM_TASKS_COMPLETED`` exit handlers;
* executor-input/-output JSON contract per step (:mod:`mipipe.dsl.executor_main`);
* artifacts under ``<pipeline_root>/<run_id>/<task>/<output>`` (``gs://`` roots map to
  the local object store, :mod:`mipipe.storage.gcs`);
* step caching keyed on (component spec, executor, resolved inputs), retries
  (``retryPolicy.maxRetryCount``), fail-fast: once a step fails no new step starts;
* a persisted run record (``run.json``) that :mod:`mipipe.client` reads back.
"""
from __future__ import annotations

import concurrent.futures as cf
import copy
import datetime as _dt
import hashlib
import json
import os
import subprocess
import sys
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

from mipipe.storage.gcs import gcs_root, uri_to_local_path
from . import cel

__all__ = ["PipelineRunner", "run_job_spec", "RunFailed", "TERMINAL_STATES"]

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SUCCEEDED, FAILED, SKIPPED, CACHED, RUNNING, PENDING, CANCELLED = (
    "SUCCEEDED", "FAILED", "SKIPPED", "CACHED", "RUNNING", "PENDING", "CANCELLED")
TERMINAL_STATES = {SUCCEEDED, FAILED, SKIPPED, CACHED, CANCELLED}


class RunFailed(RuntimeError):
    pass


def _now() -> str:
    return _dt.datetime.now().isoformat(timespec="seconds")


def _ir_value_to_py(v: Dict[str, Any]) -> Any:
    if "doubleValue" in v:
        return float(v["doubleValue"])
    if "intValue" in v:
        return int(v["intValue"])
    return v.get("stringValue")


def _py_to_ir(v: Any, ptype: str) -> Dict[str, Any]:
    if ptype == "INT":
        return {"intValue": str(int(v))}
    if ptype == "DOUBLE":
        return {"doubleValue": float(v)}
    if isinstance(v, (dict, list, bool)):
        return {"stringValue": json.dumps(v)}
    return {"stringValue": str(v)}


class PipelineRunner:
    def __init__(self, job_spec: Dict[str, Any], pipeline_root: Optional[str] = None,
                 parameter_values: Optional[Dict[str, Any]] = None,
                 run_id: Optional[str] = None, enable_caching: Optional[bool] = None,
                 max_parallel: int = 4, env: Optional[Dict[str, str]] = None,
                 echo_logs: bool = True):
        if "pipelineSpec" not in job_spec:
            job_spec = {"pipelineSpec": job_spec, "runtimeConfig": {}}
        self.spec = job_spec["pipelineSpec"]
        self.runtime = job_spec.get("runtimeConfig", {}) or {}
        self.pipeline_name = self.spec["pipelineInfo"]["name"]
        root = pipeline_root or self.runtime.get("gcsOutputDirectory")
        if not root:
            root = "gs://mipipe-default/pipeline_root"
        self.pipeline_root = root.rstrip("/")
        ts = _dt.datetime.now().strftime("%Y%m%d%H%M%S")
        self.run_id = run_id or f"{self.pipeline_name}-{ts}"
        self.run_dir = uri_to_local_path(f"{self.pipeline_root}/{self.run_id}")
        os.makedirs(self.run_dir, exist_ok=True)
        self.enable_caching = enable_caching
        self.max_parallel = max(1, int(max_parallel))
        self.extra_env = dict(env or {})
        self.echo_logs = echo_logs
        self._lock = threading.Lock()
        self._failed = threading.Event()
        self.tasks: Dict[str, Dict[str, Any]] = {}
        self.state = "PIPELINE_STATE_PENDING"
        # resolve root parameters: defaults from runtimeConfig, then overrides
        root_defs = (self.spec["root"].get("inputDefinitions") or {}).get("parameters", {})
        params: Dict[str, Dict[str, Any]] = dict(self.runtime.get("parameters") or {})
        for k, v in (parameter_values or {}).items():
            if k not in root_defs:
                raise ValueError(f"unknown pipeline parameter {k!r}; known: {sorted(root_defs)}")
            params[k] = _py_to_ir(v, root_defs[k]["type"])
        missing = [k for k in root_defs if k not in params]
        if missing:
            raise ValueError(f"pipeline parameters without value: {missing}")
        self.root_params = params
        self.cache_dir = os.environ.get("MIPIPE_CACHE_DIR",
                                        os.path.join(os.path.dirname(gcs_root()), "cache"))

    # ------------------------------------------------------------------ record
    def _record(self, path: str, **kw) -> None:
        with self._lock:
            rec = self.tasks.setdefault(path, {"state": PENDING})
            rec.update(kw)
            self._save()

    def _save(self) -> None:
        doc = {"name": self.run_id, "pipeline": self.pipeline_name, "state": self.state,
               "pipelineRoot": self.pipeline_root, "runtimeParameters": self.root_params,
               "tasks": self.tasks, "updated": _now()}
        tmp = os.path.join(self.run_dir, "run.json.tmp")
        with open(tmp, "w") as f:
            json.dump(doc, f, indent=2, sort_keys=True)
        os.replace(tmp, os.path.join(self.run_dir, "run.json"))

    # ------------------------------------------------------------------ run
    def run(self) -> Dict[str, Any]:
        self.state = "PIPELINE_STATE_RUNNING"
        self._save()
        t0 = time.time()
        try:
            self._run_dag(self.spec["root"]["dag"], {"parameters": self.root_params,
                                                     "artifacts": {}}, prefix="")
        finally:
            failed = any(r["state"] == FAILED for r in self.tasks.values())
            self.state = "PIPELINE_STATE_FAILED" if failed else "PIPELINE_STATE_SUCCEEDED"
            with self._lock:
                self._save()
        result = {"name": self.run_id, "state": self.state, "tasks": self.tasks,
                  "run_dir": self.run_dir, "wall_s": time.time() - t0}
        return result

    def _component(self, name: str) -> Dict[str, Any]:
        return self.spec["components"][name]

    def _resolve_inputs(self, task: Dict[str, Any], scope: Dict[str, Any],
                        sibling_outputs: Dict[str, Dict[str, Any]]):
        params, arts = {}, {}
        ins = task.get("inputs", {})
        for name, ref in (ins.get("parameters") or {}).items():
            if "runtimeValue" in ref:
                params[name] = ref["runtimeValue"]["constantValue"]
            elif "componentInputParameter" in ref:
                params[name] = scope["parameters"][ref["componentInputParameter"]]
            elif "taskOutputParameter" in ref:
                r = ref["taskOutputParameter"]
                params[name] = sibling_outputs[r["producerTask"]]["parameters"][r["outputParameterKey"]]
            else:
                raise ValueError(f"unsupported parameter ref {ref}")
        for name, ref in (ins.get("artifacts") or {}).items():
            if "taskOutputArtifact" in ref:
                r = ref["taskOutputArtifact"]
                arts[name] = sibling_outputs[r["producerTask"]]["artifacts"][r["outputArtifactKey"]]
            elif "componentInputArtifact" in ref:
                arts[name] = scope["artifacts"][ref["componentInputArtifact"]]
            else:
                raise ValueError(f"unsupported artifact ref {ref}")
        return params, arts

    def _run_dag(self, dag: Dict[str, Any], scope: Dict[str, Any], prefix: str) -> Dict[str, Any]:
        """Dependency-ordered execution of one (sub-)DAG on the worker pool; the state machine
        (ready / cancel / fail-fast) is the native DagScheduler (csrc/runtime/dag.cpp) or its
        Python twin :class:`_PyDag`."""
        tasks = dag.get("tasks", {})
        names = list(tasks)
        pos = {n: i for i, n in enumerate(names)}
        deps = [[pos[d] for d in tasks[n].get("dependentTasks", [])] for n in names]
        always = [((tasks[n].get("triggerPolicy") or {}).get("strategy")
                   == "ALL_UPSTREAM_TASKS_COMPLETED") for n in names]
        from mipipe.runtime import runtime, runtime_available
        sched = (runtime().DagScheduler(len(names), deps, always, True) if runtime_available()
                 else _PyDag(len(names), deps, always, True))
        code = {SUCCEEDED: 2, CACHED: 3, SKIPPED: 4, FAILED: 5}
        outputs: Dict[str, Dict[str, Any]] = {}
        for n in names:
            self._record(prefix + n, state=PENDING)
        futures: Dict[cf.Future, str] = {}
        with cf.ThreadPoolExecutor(max_workers=self.max_parallel) as pool:
            while True:
                if self._failed.is_set():
                    sched_fail_fast(sched)
                for i in sched.next_ready():
                    n = names[i]
                    fut = pool.submit(self._run_task, n, tasks[n], scope, outputs, prefix)
                    futures[fut] = n
                for i in sched.take_cancelled():
                    self._record(prefix + names[i], state=CANCELLED)
                if not futures:
                    if sched.finished():
                        break
                    raise RunFailed(f"DAG deadlock in {prefix or 'root'}: {sched.states()}")
                done, _ = cf.wait(list(futures), return_when=cf.FIRST_COMPLETED)
                for fut in done:
                    n = futures.pop(fut)
                    try:
                        st, out = fut.result()
                    except Exception as e:  # orchestrator-side error
                        st, out = FAILED, {"parameters": {}, "artifacts": {}}
                        self._record(prefix + n, state=FAILED, error=repr(e))
                    outputs[n] = out
                    sched.complete(pos[n], code.get(st, 5))
                    if st == FAILED:
                        self._failed.set()
        return outputs

    def _run_task(self, name: str, task: Dict[str, Any], scope, sibling_outputs, prefix):
        path = prefix + name
        params, arts = self._resolve_inputs(task, scope, sibling_outputs)
        cond = (task.get("triggerPolicy") or {}).get("condition")
        if cond:
            ok = cel.evaluate(cond, params)
            if not ok:
                self._record(path, state=SKIPPED, condition=cond, conditionResult=False)
                return SKIPPED, {"parameters": {}, "artifacts": {}}
        comp = self._component(task["componentRef"]["name"])
        if "dag" in comp:
            self._record(path, state=RUNNING, start=_now())
            inner = self._run_dag(comp["dag"], {"parameters": params, "artifacts": arts},
                                  prefix=path + "/")
            failed = any(self.tasks[path + "/" + k]["state"] == FAILED for k in comp["dag"]["tasks"])
            st = FAILED if failed else SUCCEEDED
            self._record(path, state=st, end=_now())
            return st, {"parameters": {}, "artifacts": {}, "inner": inner}
        executor = self.spec["deploymentSpec"]["executors"][comp["executorLabel"]]
        if "importer" in executor:
            uri = _ir_value_to_py(params["uri"])
            schema = executor["importer"]["typeSchema"]["schemaTitle"]
            art = {"name": f"{self.run_id}/{path}/artifact", "uri": uri,
                   "type": {"schemaTitle": schema},
                   "metadata": executor["importer"].get("metadata", {})}
            self._record(path, state=SUCCEEDED, start=_now(), end=_now(),
                         outputs={"artifacts": {"artifact": [art]}})
            return SUCCEEDED, {"parameters": {}, "artifacts": {"artifact": [art]}}
        return self._run_container(path, task, comp, executor["container"], params, arts)

    def _cache_key(self, comp, container, params, arts) -> str:
        h = hashlib.sha256()
        h.update(json.dumps(comp, sort_keys=True).encode())
        h.update(json.dumps(container, sort_keys=True).encode())
        h.update(json.dumps(params, sort_keys=True).encode())
        h.update(json.dumps({k: [a["uri"] for a in v] for k, v in arts.items()},
                            sort_keys=True).encode())
        return h.hexdigest()

    def _run_container(self, path, task, comp, container, params, arts):
        task_dir = os.path.join(self.run_dir, path.replace("/", os.sep))
        os.makedirs(task_dir, exist_ok=True)
        out_defs = comp.get("outputDefinitions", {})
        exec_outputs: Dict[str, Any] = {"parameters": {}, "artifacts": {},
                                        "outputFile": os.path.join(task_dir, "executor_output.json")}
        out_arts = {}
        for oname, odef in (out_defs.get("artifacts") or {}).items():
            uri = f"{self.pipeline_root}/{self.run_id}/{path}/{oname}"
            a = {"name": f"{self.run_id}/{path}/{oname}", "uri": uri,
                 "type": {"schemaTitle": odef["artifactType"]["schemaTitle"]}, "metadata": {}}
            out_arts[oname] = [a]
            exec_outputs["artifacts"][oname] = {"artifacts": [a]}
        for pname in (out_defs.get("parameters") or {}):
            exec_outputs["parameters"][pname] = {
                "outputFile": os.path.join(task_dir, "parameters", pname)}
        executor_input = {"inputs": {"parameters": params,
                                     "artifacts": {k: {"artifacts": v} for k, v in arts.items()}},
                          "outputs": exec_outputs}
        caching = task.get("cachingOptions", {}).get("enableCache", True)
        if self.enable_caching is not None:
            caching = self.enable_caching
        key = self._cache_key(comp, container, params, arts)
        cache_file = os.path.join(self.cache_dir, key + ".json")
        if caching and os.path.isfile(cache_file):
            with open(cache_file) as f:
                cached = json.load(f)
            if all(os.path.exists(uri_to_local_path(a["uri"]))
                   for lst in cached["artifacts"].values() for a in lst):
                self._record(path, state=CACHED, start=_now(), end=_now(), cacheKey=key,
                             outputs=cached)
                return CACHED, cached
        retries = int((task.get("retryPolicy") or {}).get("maxRetryCount", 0))
        opts = task.get("mipipeOptions", {})
        env = dict(os.environ)
        env.update(self.extra_env)
        env.update(opts.get("env", {}))
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env["MIPIPE_GCS_ROOT"] = gcs_root()
        env["MIPIPE_RUN_ID"] = self.run_id
        env["MIPIPE_TASK"] = path
        cmd = [c.replace("{{$}}", json.dumps(executor_input)) for c in container["command"]]
        cmd += [c.replace("{{$}}", json.dumps(executor_input)) for c in container.get("args", [])]
        log_path = os.path.join(task_dir, "log.txt")
        attempt, rc = 0, None
        start = _now()
        while True:
            attempt += 1
            self._record(path, state=RUNNING, start=start, attempts=attempt, log=log_path)
            with open(log_path, "a") as log:
                log.write(f"=== attempt {attempt} {_now()} ===\n")
                log.flush()
                p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                     env=env, cwd=task_dir, text=True, bufsize=1,
                                     start_new_session=True)
                for line in p.stdout:
                    log.write(line)
                    if self.echo_logs:
                        sys.stdout.write(f"[{path}] {line}")
                rc = p.wait()
            if rc == 0 or attempt > retries:
                break
        if rc != 0:
            self._record(path, state=FAILED, end=_now(), exitCode=rc)
            return FAILED, {"parameters": {}, "artifacts": {}}
        produced = {"parameters": {}, "artifacts": out_arts}
        of = exec_outputs["outputFile"]
        if os.path.isfile(of):
            with open(of) as f:
                eo = json.load(f)
            produced["parameters"].update(eo.get("parameters", {}))
            for k, v in (eo.get("artifacts") or {}).items():
                if v.get("artifacts"):
                    produced["artifacts"][k] = [dict(out_arts.get(k, [{}])[0], **{
                        "metadata": v["artifacts"][0].get("metadata", {})})]
        for pname, pdef in (out_defs.get("parameters") or {}).items():
            if pname not in produced["parameters"]:
                pf = exec_outputs["parameters"][pname]["outputFile"]
                if os.path.isfile(pf):
                    with open(pf) as f:
                        produced["parameters"][pname] = _py_to_ir(f.read(), pdef["type"])
        if caching:
            os.makedirs(self.cache_dir, exist_ok=True)
            with open(cache_file + ".tmp", "w") as f:
                json.dump(produced, f)
            os.replace(cache_file + ".tmp", cache_file)
        self._record(path, state=SUCCEEDED, end=_now(), exitCode=0, outputs=produced,
                     cacheKey=key)
        return SUCCEEDED, produced


def run_job_spec(job_spec_path: str, pipeline_root: Optional[str] = None,
                 parameter_values: Optional[Dict[str, Any]] = None, **kw) -> Dict[str, Any]:
    with open(job_spec_path) as f:
        spec = json.load(f)
    return PipelineRunner(spec, pipeline_root, parameter_values, **kw).run()


def sched_fail_fast(sched) -> None:
    """A failure elsewhere in the run (another sub-DAG) cancels this DAG's pending tasks."""
    if isinstance(sched, _PyDag):
        sched.any_failed = True
    else:
        sched.mark_external_failure()


class _PyDag:
    """Pure-Python twin of the native DagScheduler (same states and semantics)."""

    PENDING, RUNNING, SUCCEEDED, CACHED, SKIPPED, FAILED, CANCELLED = range(7)

    def __init__(self, n, deps, always_run, fail_fast=True):
        self.n, self.deps, self.always, self.fail_fast = n, deps, always_run, fail_fast
        self.state = [self.PENDING] * n
        self.cancelled = []
        self.any_failed = False
        indeg = [len(d) for d in deps]
        children = [[] for _ in range(n)]
        for i, ds in enumerate(deps):
            for d in ds:
                children[d].append(i)
        q = [i for i in range(n) if indeg[i] == 0]
        for i in q:
            for c in children[i]:
                indeg[c] -= 1
                if indeg[c] == 0:
                    q.append(c)
        if len(q) != n:
            raise ValueError("pipeline DAG has a cycle")
        self.topo = q

    def next_ready(self):
        out, changed = [], True
        while changed:
            changed = False
            for i in self.topo:
                if self.state[i] != self.PENDING:
                    continue
                ds = self.deps[i]
                if any(self.state[d] < self.SUCCEEDED for d in ds):
                    continue
                up_failed = any(self.state[d] in (self.FAILED, self.CANCELLED) for d in ds)
                if not self.always[i] and (up_failed or (self.fail_fast and self.any_failed)):
                    self.state[i] = self.CANCELLED
                    self.cancelled.append(i)
                    changed = True
                    continue
                self.state[i] = self.RUNNING
                out.append(i)
        return out

    def complete(self, i, st):
        if self.state[i] != self.RUNNING:
            raise RuntimeError("complete() on a task that is not running")
        self.state[i] = st
        if st == self.FAILED:
            self.any_failed = True

    def take_cancelled(self):
        r, self.cancelled = self.cancelled, []
        return r

    def finished(self):
        return all(s >= self.SUCCEEDED for s in self.state)

    def states(self):
        return list(self.state)
