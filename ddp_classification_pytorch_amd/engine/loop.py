"""Generic epoch loop for the single-loss classification workloads
(BASELINE ``train_and_valid`` BASELINE/main.py:258-314, ARCFACE loop
ARCFACE/arc_main.py:302-414, CDR ``train``/``evaluate`` CDR/main.py:218-283).

Differences from the reference, all deliberate:
* metrics (loss sum, top-1, top-3, count) accumulate on the device every
  step and are reduced with ONE all_reduce per log interval / epoch, so they
  are exact over the global batch (the reference multiplies rank-0 counts by
  world_size, BASELINE/main.py:247-249) and cost no per-step host syncs;
* validation excludes the DistributedSampler padding duplicates;
* ``set_epoch`` is always called (ARCFACE forgets it);
* checkpoints are state_dicts written once by rank 0 (``last.pth`` /
  ``best.pth``) and ``--resume`` restores model/optimizer/scheduler/epoch/RNG;
* ``--fail-at-step`` injects a failure for resume testing; ``--auto-resume``
  restarts from ``last.pth`` when it exists (a relaunch after a failure continues);
* ``--warmup-iters`` ramps the learning rate linearly per iteration from 1e-6
  (BASELINE ``WarmUp``, BASELINE/main.py:170-197; dead code in the reference,
  wired here for every workload that goes through this loop);
* GPU step time from HIP events (``gpu_ms_per_step`` in the JSONL log, no host
  sync beyond the log interval's), a per-rank heartbeat file
  (``heartbeat_rank<r>.txt``: wall time, step, loss every ``--heartbeat-every``
  steps, so a hung or dead rank is visible), and ``--profile``: a torch.profiler
  (roctracer) trace of a few steps of the first epoch into ``<out-dir>/profile``.
"""
from __future__ import annotations

import math
import os
import time

import torch
import torch.distributed as dist

from ..ops import functional as Fn
from ..optim.schedulers import LinearWarmup
from .checkpoint import load_checkpoint, save_checkpoint
from .logger import MetricsLogger


class InjectedFailure(RuntimeError):
    pass


def _allreduce(t):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return t


def _check_transports():
    """Fail loudly if a SyncBN peer exchange timed out (parallel/peer.py: its results are NaN);
    a no-op unless the peer transport is on.  Called where the loop synchronises anyway."""
    if torch.cuda.is_available():
        from ..parallel import peer

        peer.check_all()


def valid_count(sampler, n_total):
    """Samples of this rank that are not DistributedSampler padding."""
    if sampler is None or not hasattr(sampler, "world"):
        return n_total
    return max(0, math.ceil((sampler.n - sampler.rank) / sampler.world))


class ClassificationLoop:
    """``forward_train(batch) -> (loss, rank)``; ``forward_eval(batch) -> (loss_rows, rank)``;
    optional ``post_backward()`` (e.g. CDR gradient masking) and ``epoch_hook(epoch)``."""

    def __init__(self, args, rt, models: dict, optimizer, scheduler, train_data, val_data, forward_train,
                 forward_eval, post_backward=None, logger: MetricsLogger = None, scheduler_before_epoch=False,
                 train_modules=None):
        self.args, self.rt = args, rt
        self.models, self.optimizer, self.scheduler = models, optimizer, scheduler
        self.train_data, self.val_data = train_data, val_data
        self.forward_train, self.forward_eval = forward_train, forward_eval
        self.post_backward = post_backward
        self.logger = logger or MetricsLogger(args.out_dir if rt.is_main else None)
        self.scheduler_before_epoch = scheduler_before_epoch  # CDR steps its scheduler before training (:365-366)
        self.train_modules = train_modules or list(models.values())
        self.start_epoch, self.global_step, self.best = 0, 0, -1.0
        self.warmup = None
        self._warmup_state = None  # LinearWarmup.state_dict() from a resumed checkpoint

    # ------------------------------------------------------------------ persistence
    def _ckpt(self, name):
        return os.path.join(self.args.out_dir, name)

    def maybe_resume(self):
        path = self.args.resume
        if path is None and os.path.exists(self._ckpt("last.pth")) and getattr(self.args, "auto_resume", False):
            path = self._ckpt("last.pth")
        if not path:
            return
        # CPU map: the RNG ByteTensors must stay host tensors for set_rng_state; load_state_dict
        # copies model / optimizer state onto the parameters' device
        extra = load_checkpoint(path, self.models, {"opt": self.optimizer},
                                {"sched": self.scheduler} if self.scheduler is not None else None,
                                map_location="cpu")
        self.start_epoch = int(extra.get("epoch", -1)) + 1
        self.global_step = int(extra.get("global_step", 0))
        self.best = float(extra.get("best", -1.0))
        self._warmup_state = extra.get("warmup")
        self.logger.line(f"resumed from {path}: epoch {self.start_epoch}, step {self.global_step}")

    def save(self, epoch, val_top1):
        kw = dict(epoch=epoch, global_step=self.global_step, best=max(self.best, val_top1),
                  warmup=self.warmup.state_dict() if self.warmup is not None else None,
                  config={k: v for k, v in vars(self.args).items() if isinstance(v, (int, float, str, bool, list))})
        sched = {"sched": self.scheduler} if self.scheduler is not None else None
        save_checkpoint(self._ckpt("last.pth"), self.models, {"opt": self.optimizer}, sched, **kw)
        if val_top1 > self.best:
            self.best = val_top1
            save_checkpoint(self._ckpt("best.pth"), self.models, {"opt": self.optimizer}, sched, **kw)

    # ------------------------------------------------------------------ epochs
    def _train_step(self, *batch):
        loss, rank = self.forward_train(batch)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        if self.post_backward is not None:
            self.post_backward()
        self.optimizer.step()
        # detached: a loss kept alive until the next step would keep this step's autograd graph --
        # and with it the parameters' AccumulateGrad nodes, bound to this step's stream -- alive
        # into a HIP-graph capture, whose gradient accumulation would then sync with that stream
        return loss.detach(), rank

    def _setup_graph(self):
        """--graph: single-process GPU runs replay the whole step as a HIP graph (engine/graph.py),
        recaptured at every epoch start (the learning rate is a captured kernel argument) and
        after the LR warm-up (its steps run eagerly: the LR changes every iteration)."""
        a = self.args
        self._grapher = None
        graph_safe = not any(isinstance(m, torch.nn.parallel.DistributedDataParallel) for m in self.train_modules)
        if getattr(a, "graph", False) and self.rt.device.type == "cuda" and (self.rt.world == 1 or graph_safe):
            from .graph import HostCounters, StepGrapher

            mods = list(self.models.values()) + list(self.train_modules)
            self._grapher = StepGrapher(self._train_step, warmup=2, counters=HostCounters(mods, [self.optimizer]))

    def _setup_warmup(self):
        """The ramp's target is the configured ``--lr`` (or the scheduler's base LR), never the
        optimizer's current LR: a checkpoint written mid-ramp restores a partial-ramp LR into the
        optimizer, and ramping towards that would leave a resumed run below the uninterrupted one."""
        iters = int(getattr(self.args, "warmup_iters", 0) or 0)
        if iters > 0 and self.global_step < iters and self.warmup is None:
            target = getattr(self.args, "lr", None)
            if target is None and self.scheduler is not None and getattr(self.scheduler, "base_lrs", None):
                target = self.scheduler.base_lrs[0]
            if target is None:
                target = self.optimizer.param_groups[0].get("initial_lr", self.optimizer.param_groups[0]["lr"])
            self.warmup = LinearWarmup(self.optimizer, iters, float(target), start_lr=1e-6)
            self.warmup.n = self.global_step  # resumed mid-warm-up: continue the ramp
            if self._warmup_state is not None and self._warmup_state.get("iters") == iters:
                self.warmup.load_state_dict(self._warmup_state)

    def _heartbeat(self, epoch):
        """Host-only (no device sync): wall time and step, so a stalled rank stops advancing."""
        every = int(getattr(self.args, "heartbeat_every", 0) or 0)
        if not every or self.global_step % every or not self.args.out_dir:
            return
        os.makedirs(self.args.out_dir, exist_ok=True)
        with open(os.path.join(self.args.out_dir, f"heartbeat_rank{self.rt.rank}.txt"), "a") as f:
            f.write(f"{time.time():.3f} rank {self.rt.rank} epoch {epoch} step {self.global_step}\n")

    def train_epoch(self, epoch):
        a, dev = self.args, self.rt.device
        if not hasattr(self, "_grapher"):
            self._setup_graph()
        if self._grapher is not None:
            self._grapher.reset()  # the epoch's learning rate is baked into the captured step
        self._setup_warmup()
        prof = None
        if getattr(a, "profile", False) and epoch == self.start_epoch and self.rt.is_main:
            prof = torch.profiler.profile(
                activities=[torch.profiler.ProfilerActivity.CPU] +
                ([torch.profiler.ProfilerActivity.CUDA] if dev.type == "cuda" else []),
                schedule=torch.profiler.schedule(wait=1, warmup=1, active=4, repeat=1))
            prof.__enter__()
        timing = dev.type == "cuda"
        ev0 = torch.cuda.Event(enable_timing=True) if timing else None
        ev1 = torch.cuda.Event(enable_timing=True) if timing else None
        win_steps = 0
        for m in self.train_modules:
            m.train()
        sampler = getattr(self.train_data, "sampler", None)
        if sampler is not None and hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        acc = torch.zeros(4, dtype=torch.float64, device=dev)  # loss*B, top1, top3, count
        win = torch.zeros(4, dtype=torch.float64, device=dev)
        n_steps = len(self.train_data)
        if a.max_steps_per_epoch:
            n_steps = min(n_steps, a.max_steps_per_epoch)
        t0 = t_win = time.time()
        for i, batch in enumerate(self.train_data):
            if i >= n_steps:
                break
            if a.fail_at_step is not None and self.global_step == a.fail_at_step:
                raise InjectedFailure(f"injected failure at global step {self.global_step}")
            if timing and win_steps == 0:
                ev0.record()
            in_warmup = self.warmup is not None and not self.warmup.done
            if in_warmup:
                self.warmup.step()
            if self._grapher is not None and not in_warmup:
                loss, rank = self._grapher(*batch)
            elif self._grapher is not None:
                loss, rank = self._grapher.eager(*batch)  # the grapher's side stream, as its own warm-up
                if self.warmup.done:
                    self._grapher.reset()  # capture at the final warm-up learning rate
            else:
                loss, rank = self._train_step(*batch)
            win_steps += 1
            if prof is not None:
                prof.step()
            B = rank.numel()
            # one launch, no host->device copy (a torch.tensor(B, device=...) here synchronised the
            # stream every step); the window folds into the epoch totals at each log point
            Fn.metric_accum(win, loss, B, rank, B)
            self.global_step += 1
            self._heartbeat(epoch)
            if (i + 1) % a.log_interval == 0 or i + 1 == n_steps:
                gpu_ms = None
                if timing:
                    ev1.record()
                acc += win
                w = _allreduce(win.clone()).tolist()
                if timing:
                    ev1.synchronize()
                    gpu_ms = ev0.elapsed_time(ev1) / max(win_steps, 1)
                _check_transports()
                now = time.time()
                win_ips = win_steps * B * self.rt.world / max(now - t_win, 1e-9)  # window wall rate (synced above)
                t_win = now
                win_steps = 0
                dt = now - t0
                eta = dt / (i + 1) * (n_steps - i - 1)
                lr = self.optimizer.param_groups[0]["lr"]
                self.logger.progress(
                    f"Epoch [{epoch + 1}/{a.epochs}] Iter [{i + 1}/{n_steps}] loss {w[0] / max(w[3], 1):.4f} "
                    f"top1 {100 * w[1] / max(w[3], 1):.2f} top3 {100 * w[2] / max(w[3], 1):.2f} lr {lr:.3g} "
                    f"{(i + 1) * B * self.rt.world / max(dt, 1e-9):.0f} img/s "
                    f"eta {eta:.0f}s")
                self.logger.log("train_iter", epoch=epoch, step=self.global_step, loss=w[0] / max(w[3], 1),
                                top1=w[1] / max(w[3], 1), top3=w[2] / max(w[3], 1), lr=lr, gpu_ms_per_step=gpu_ms,
                                img_per_s=win_ips)
                win.zero_()
        if prof is not None:
            prof.__exit__(None, None, None)
            pdir = os.path.join(a.out_dir, "profile")
            os.makedirs(pdir, exist_ok=True)
            with open(os.path.join(pdir, "steps.txt"), "w") as f:
                f.write(prof.key_averages().table(sort_by="self_cuda_time_total" if timing else "self_cpu_time_total",
                                                  row_limit=60))
            prof.export_chrome_trace(os.path.join(pdir, "trace.json"))
        tot = _allreduce(acc).tolist()
        _check_transports()
        self.logger.progress("", end="\n")
        n = max(tot[3], 1)
        return {"loss": tot[0] / n, "top1": tot[1] / n, "top3": tot[2] / n, "count": tot[3],
                "time": time.time() - t0}

    @torch.no_grad()
    def evaluate(self):
        for m in self.train_modules:
            m.eval()
        dev = self.rt.device
        sampler = getattr(self.val_data, "sampler", None)
        left = valid_count(sampler, float("inf"))
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        for batch in self.val_data:
            loss_rows, rank = self.forward_eval(batch)
            B = rank.numel()
            k = int(min(B, left))
            left -= k
            if k <= 0:
                continue
            Fn.metric_accum(acc, loss_rows[:k], 1.0, rank, k)
        tot = _allreduce(acc).tolist()
        n = max(tot[3], 1)
        return {"loss": tot[0] / n, "top1": tot[1] / n, "top3": tot[2] / n, "count": tot[3]}

    def run(self):
        a = self.args
        self.maybe_resume()
        for epoch in range(self.start_epoch, a.epochs):
            if self.scheduler is not None and self.scheduler_before_epoch:
                self.scheduler.step()
            tr = self.train_epoch(epoch)
            self.logger.log("train_epoch", epoch=epoch, **tr)
            va = {"top1": -1.0}
            if self.val_data is not None and ((epoch + 1) % a.eval_every == 0 or epoch + 1 == a.epochs):
                va = self.evaluate()
                self.logger.log("val", epoch=epoch, **va)
                self.logger.line(f"VAL Epoch {epoch + 1}: loss {va['loss']:.4f} top1 {100 * va['top1']:.3f} "
                                 f"top3 {100 * va['top3']:.3f} (n={int(va['count'])}) | train loss {tr['loss']:.4f} "
                                 f"top1 {100 * tr['top1']:.3f} ({tr['time']:.1f}s)")
            if self.scheduler is not None and not self.scheduler_before_epoch:
                self.scheduler.step()
            if (epoch + 1) % a.save_every == 0 or epoch + 1 == a.epochs:
                self.save(epoch, va["top1"])
        self.logger.dump_history()
        return self.best
