"""Training on the HIP engine: model_fn's TRAIN / EVAL branches (code/utils/generate_model.py:697-830,
"GM") and the loop of train_and_evaluate (code/utils/framework_operations.py:108-166, "FO").

* loss: ``learning_options.loss`` (MeanSquaredError, GM:745-753) over the batch's concatenated
  flat predictions, plus the Dense l2 kernel regularizers (AUX:833-834).  The engine computes
  it (``ign_mse_loss``, ``ign_l2_loss``).
* gradients: ``ign_backward``, the HIP backward of the whole forward (tf.gradients, GM:790).
* optimizer: ``learning_options.optimizer`` (GM:797-818).  Only Adam is lowered (``ign_adam_step``,
  Keras semantics); the learning rate is a float or an ExponentialDecay schedule evaluated at
  ``iterations`` (the global step, GM:816).
* data parallel: with torch.distributed initialised, every rank trains on its own batches and
  the gradient is averaged with one all-reduce (RCCL on GPUs) before the update.
* eval metrics (GM:755-785): label/prediction mean, MAE, MRE and the batch-mean r-squared
  (GM:201-216), after denormalisation, plus the mean loss.
"""

from __future__ import annotations

import math
import os
import time

import numpy as np

from .engine import UnsupportedModel
from .generate_model import ComnetModel, _resolve

SUPPORTED_LOSSES = ("MeanSquaredError",)


class LearningRate:
    """``optimizer.learning_rate`` or ``optimizer.schedule`` (Keras ExponentialDecay)."""

    def __init__(self, opt: dict):
        sched = opt.get("schedule")
        self.kind = "constant"
        self.lr0 = float(opt.get("learning_rate", 0.001))
        if sched is not None:
            sched = dict(sched)
            kind = sched.pop("type")
            if kind != "ExponentialDecay":
                raise UnsupportedModel("learning-rate schedule %r is not lowered (ExponentialDecay only)" % kind)
            self.kind = kind
            self.lr0 = float(sched["initial_learning_rate"])
            self.decay_steps = float(sched["decay_steps"])
            self.decay_rate = float(sched["decay_rate"])
            # Keras tests `if self.staircase:`; a JSON string such as "True" (QSJ:204) or even
            # "False" is truthy there
            self.staircase = bool(sched.get("staircase", False))

    def __call__(self, step: int) -> float:
        if self.kind == "constant":
            return self.lr0
        p = step / self.decay_steps
        if self.staircase:
            p = math.floor(p)
        return self.lr0 * self.decay_rate ** p


class Trainer:
    def __init__(self, model_info, params: dict | None = None, device: int = 0, seed: int = 0, dist=None):
        import torch
        self.torch = torch
        loss = model_info.get_loss()
        if loss not in SUPPORTED_LOSSES:
            raise UnsupportedModel("loss %r is not lowered (%s)" % (loss, ", ".join(SUPPORTED_LOSSES)))
        opt = dict(model_info.get_optimizer())
        if opt.get("type") != "Adam":
            raise UnsupportedModel("optimizer %r is not lowered (Adam only)" % opt.get("type"))
        self.lr = LearningRate(opt)
        self.beta1 = float(opt.get("beta_1", 0.9))
        self.beta2 = float(opt.get("beta_2", 0.999))
        self.epsilon = float(opt.get("epsilon", 1e-7))
        self.model_info = model_info
        torch.cuda.set_device(device)
        self.model = ComnetModel(model_info, device=device, params=params, seed=seed)
        eng = self.model.engine
        eng.set_stream(torch.cuda.current_stream().cuda_stream)   # torch copies / RCCL stream-ordered
        dev = torch.device("cuda", device)
        self.grads = torch.zeros(eng.n_params, dtype=torch.float32, device=dev)
        self.m = torch.zeros_like(self.grads)
        self.v = torch.zeros_like(self.grads)
        self.dpred = None
        self.device = dev
        self.dist = dist
        self.iterations = 0
        # IGN_STEP_PROF=1: host seconds per phase of train_prepared (bench.py --fresh-batches reports them)
        self.step_prof = (dict.fromkeys(("forward_enqueue", "loss_wait", "backward_enqueue", "close", "l2_wait",
                                         "steps"), 0.0) if os.environ.get("IGN_STEP_PROF") == "1" else None)
        self.output_name, _, self.output_denorm = model_info.get_output_info()

    @property
    def engine(self):
        return self.model.engine

    def _labels(self, labels):
        y = np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels])
        return self.torch.from_numpy(y).to(self.device)

    def prepare(self, features, labels):
        """The host half of a step: the batch (CSR tables, H2D copies, the training tables) and the
        device label vector.  Safe on a worker thread while the GPU runs another step (the engine
        builds batches on a non-blocking stream of the calling thread; the labels use a torch
        stream of their own)."""
        b = self.model.batch(features)
        try:
            b.enable_training()
            y = np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels])
            if y.size != b.predictions * b.output_units:
                raise ValueError("labels hold %d values for %d predictions" % (y.size, b.predictions * b.output_units))
            torch = self.torch
            with torch.cuda.device(self.device):
                s = torch.cuda.Stream(self.device)
                with torch.cuda.stream(s):
                    yd = torch.from_numpy(y).pin_memory().to(self.device, non_blocking=True)
                s.synchronize()
        except BaseException:
            b.close()
            raise
        return b, yd

    def train_step(self, features: list, labels: list) -> dict:
        """One optimizer step on a batch of graphs (model_fn TRAIN, GM:712-830)."""
        return self.train_prepared(*self.prepare(features, labels))

    def train_prepared(self, b, y, want_loss: bool = True) -> dict:
        """One optimizer step on a batch made by ``prepare`` (closed here).  ``want_loss=False``: the
        step is only enqueued -- no host wait for the loss or the regularisation term (the returned
        dict has None for them), so the next step's host work overlaps this one on the GPU; the
        training loop asks for them on the steps it logs (tf.estimator computes the loss every step
        but only the logged steps reach the host)."""
        prof = self.step_prof
        tick = time.perf_counter if prof is not None else None
        t0 = tick() if tick else 0.0
        # y was made on a builder's stream: without a host wait in this step, its memory must not
        # return to that stream's pool before the step has read it
        y.record_stream(self.torch.cuda.current_stream(y.device))
        try:
            b.forward_train(to_host=False)
            if tick:
                t1 = tick()
                prof["forward_enqueue"] += t1 - t0
            dpred = self.torch.empty_like(y)
            loss = self.engine.mse_loss(b.predictions_ptr(), y, dpred, want_loss=want_loss)
            if tick:
                t2 = tick()
                prof["loss_wait"] += t2 - t1
            b.backward(dpred, self.grads)
            if tick:
                t3 = tick()
                prof["backward_enqueue"] += t3 - t2
            if self.dist is not None and self.dist.is_initialized() and self.dist.get_world_size() > 1:
                if self.dist.get_backend() == "gloo":   # CPU collectives (tests, rehearsals): host-staged
                    g = self.grads.cpu()
                    self.dist.all_reduce(g)
                    self.grads.copy_(g)
                else:                                   # RCCL over xGMI
                    self.dist.all_reduce(self.grads)
                self.grads /= self.dist.get_world_size()
            lr = self.lr(self.iterations)
            self.engine.adam_step(self.grads, self.m, self.v, self.iterations, lr, self.beta1, self.beta2, self.epsilon)
            self.iterations += 1
        finally:
            if tick:
                t4 = tick()
            b.close()
            if tick:
                t5 = tick()
                prof["close"] += t5 - t4
        reg = self.engine.l2_loss() if want_loss else None
        if tick:
            prof["l2_wait"] += tick() - t5
            prof["steps"] += 1
        return {"loss": loss, "regularization_loss": reg, "total_loss": loss + reg if want_loss else None,
                "learning_rate": lr, "step": self.iterations}

    def _denorm(self, v):
        if self.output_denorm is None or str(self.output_denorm) == "None":
            return v
        try:
            return _resolve(self.output_denorm)(v, self.output_name)
        except KeyError:
            return v

    def evaluate(self, batches) -> dict:
        """model_fn EVAL (GM:755-785) over an iterable of (features, labels) batches."""
        labels_all, preds_all, losses, r2 = [], [], [], []
        for features, labels in batches:
            b = self.model.batch(features)
            try:
                p = b.forward().reshape(-1).astype(np.float64)
            finally:
                b.close()
            y = np.concatenate([np.asarray(l, np.float64).reshape(-1) for l in labels])
            losses.append(float(np.mean((y - p) ** 2)))
            yd = np.asarray(self._denorm(y), np.float64)
            pd = np.asarray(self._denorm(p), np.float64)
            labels_all.append(yd)
            preds_all.append(pd)
            tot = np.sum((yd - yd.mean()) ** 2)
            r2.append(1.0 - np.sum((yd - pd) ** 2) / tot if tot > 0 else float("nan"))
        y = np.concatenate(labels_all)
        p = np.concatenate(preds_all)
        with np.errstate(divide="ignore", invalid="ignore"):
            rel = np.where(y != 0, np.abs(y - p) / np.abs(y), 0.0)   # div_no_nan
        return {"loss": float(np.mean(losses)), "label/mean": float(y.mean()), "prediction/mean": float(p.mean()),
                "mae": float(np.mean(np.abs(y - p))), "mre": float(rel.mean()), "r-squared": float(np.nanmean(r2)),
                "samples": int(len(losses))}

    def params(self) -> dict:
        return self.engine.get_params()

    def prefetch(self, jobs, depth: int = 2, workers: int = 1, load=None) -> "BatchPrefetcher":
        return BatchPrefetcher(self, jobs, depth, workers, load)

    def set_params(self, params: dict):
        self.model.set_params(params)


def builder_cpus(workers: int) -> list:
    """CPU sets for ``workers`` batch-builder threads (IGN_PIN_BUILDERS=1; default off): two CPUs each,
    consecutive ones of the NUMA node the calling thread runs on, within the process's affinity
    (local rank r of a multi-rank node takes the r-th slice).
    A builder's index tables are memory-bound host work; a thread the scheduler moved across CCDs
    and NUMA nodes between batches ran the ordered MP's message lists at 20-21 ms instead of
    10 ms pinned (one builder, `r06_c22.sh`).  With eight builders on a shared host it measured
    slower (24.0-26.6 against 19.0-23.9 ms per fresh-batch step, `r06_c23.sh`: the low CPUs it
    picks are other tenants' too), hence off by default.  Empty sets (no pinning) when the switch
    is off, the topology is unreadable, or the node has fewer than one CPU per builder."""
    if os.environ.get("IGN_PIN_BUILDERS", "0") != "1" or not hasattr(os, "sched_getaffinity"):
        return [set() for _ in range(workers)]
    try:
        allowed = os.sched_getaffinity(0)
        with open("/proc/self/stat") as f:
            cur = int(f.read().rsplit(")", 1)[1].split()[36])   # field 39: the CPU last run on
        node = set(allowed)
        for path in sorted(os.listdir("/sys/devices/system/node")):
            if not path.startswith("node"):
                continue
            cpus = set()
            with open("/sys/devices/system/node/%s/cpulist" % path) as f:
                for part in f.read().strip().split(","):
                    lo, _, hi = part.partition("-")
                    cpus.update(range(int(lo), int(hi or lo) + 1))
            if cur in cpus:
                node = cpus & set(allowed)
                break
    except (OSError, ValueError, IndexError):
        return [set() for _ in range(workers)]
    cand = sorted(node)
    # ranks of one node (torchrun's LOCAL_RANK) take disjoint slices; no pinning when they do not fit
    lr = int(os.environ.get("LOCAL_RANK", "0") or 0)
    per = 2 if len(cand) >= 2 * workers * (lr + 1) else 1 if len(cand) >= workers * (lr + 1) else 0
    if per == 0:
        return [set() for _ in range(workers)]
    base = lr * workers * per
    return [set(cand[base + per * i:base + per * i + per]) for i in range(workers)]


class BatchPrefetcher:
    """The training input pipeline overlapped with the GPU (the role of tf.data's
    ``map(num_parallel_calls)`` + ``prefetch``, GM:181-192).  ``workers`` threads take the next
    jobs of ``jobs`` (in order), turn each into (features, labels) with ``load`` (default: the job
    is that pair; with the native reader, ``NativeInput.load`` of a batch of sample ids) and run
    ``Trainer.prepare`` on it (the engine's host CSR build and copies, the training tables), while
    the main thread's step runs on the GPU.  At most ``depth`` batches are built ahead.  Iterating
    yields prepared (batch, labels) pairs in job order, for ``Trainer.train_prepared``; an
    exception in a worker is raised in the consumer at its position."""

    _END = object()

    def __init__(self, trainer: Trainer, jobs, depth: int = 2, workers: int = 1, load=None):
        import threading
        self.trainer = trainer
        self.jobs = iter(jobs)
        self.load = load
        self.lock = threading.Lock()          # the job iterator
        self.cv = threading.Condition()       # results by sequence number
        self.slots = threading.Semaphore(max(1, depth))
        self.results = {}
        self.issued = 0
        self.end = None                       # sequence number of the end of the jobs
        self.next_out = 0
        self.stop = threading.Event()
        cpus = builder_cpus(max(1, workers))
        self.threads = [threading.Thread(target=self._run, args=(c,), daemon=True) for c in cpus]
        for t in self.threads:
            t.start()

    def _run(self, cpus=frozenset()):
        if cpus:
            try:
                os.sched_setaffinity(0, cpus)   # this thread (Linux: pid 0 is the caller)
            except OSError:
                pass
        while True:
            while not self.slots.acquire(timeout=0.1):
                if self.stop.is_set():
                    return
            if self.stop.is_set():
                return
            with self.lock:
                if self.end is not None:
                    self.slots.release()
                    return
                k = self.issued
                try:
                    job = next(self.jobs)
                except StopIteration:
                    self.end = k
                    with self.cv:
                        self.cv.notify_all()
                    self.slots.release()
                    return
                except BaseException as e:
                    self.end = k + 1
                    job = e
                self.issued += 1
            try:
                if isinstance(job, BaseException):
                    raise job
                features, labels = self.load(job) if self.load is not None else job
                res = self.trainer.prepare(features, labels)
                # the gathered arrays are copied into the batch: drop them now, so that the native
                # reader's buffers go back to its pool before this worker's next gather
                del features, labels
            except BaseException as e:   # handed to the consumer
                res = e
            with self.cv:
                self.results[k] = res
                self.cv.notify_all()

    def __iter__(self):
        return self

    def __next__(self):
        with self.cv:
            while self.next_out not in self.results:
                if self.end is not None and self.next_out >= self.end:
                    raise StopIteration
                self.cv.wait(0.1)
            res = self.results.pop(self.next_out)
            self.next_out += 1
        self.slots.release()
        if isinstance(res, BaseException):
            raise res
        return res

    def close(self):
        self.stop.set()
        for t in self.threads:
            t.join()
        with self.cv:
            for res in self.results.values():
                if isinstance(res, tuple):
                    res[0].close()
            self.results.clear()
