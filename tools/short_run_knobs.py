"""Host-side (and launch-shape) settings on the driver's short timed region (VERDICT r03 item 1:
the K = 20 wall vs HIP-event gap).  The region is bench.timed_multi's: two
stream events around one k_step_multi launch of K ticks, then a device
synchronize.  Each setting runs in its own child process (the parent never
touches the GPU), and reports medians over reps of

  wall        the region exactly as bench.py times it
  event       its HIP-event span
  wall_poll   the same region with a busy poll of the end event before the
              synchronize (the wait spins instead of sleeping)
  empty       the two events and the synchronize alone

    python tools/short_run_knobs.py [--k 20] [--reps 40] [--only NAME,...]
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SETTINGS = {
    "default": {},
    "active_wait_1ms": {"ROC_ACTIVE_WAIT_TIMEOUT": "1000"},
    "dev_kernarg_1": {"HIP_FORCE_DEV_KERNARG": "1"},
    "dev_kernarg_0": {"HIP_FORCE_DEV_KERNARG": "0"},
    "schedule_spin": {"SK_KNOB_SCHEDULE_SPIN": "1"},
    # the kernel's own launch shape: 256-lane workgroups (a quarter of the
    # workgroups to dispatch) and the restart draw under the loads
    "block_256": {"SK_MULTI_BLOCK": "256"},
    "early_draw": {"SK_MULTI_EARLY": "1"},
    # round 6: two lanes per game and the packed resident form at the K = 20 launch
    "split_geometry": {"SK_MULTI_SPLIT": "1"},
    "packed_form": {"SK_MULTI_PACK": "1"},
    "split_prefetch1": {"SK_MULTI_SPLIT": "1", "SK_MULTI_PREFETCH": "1"},
}


def child(k, reps, envs):
    if os.environ.get("SK_KNOB_SCHEDULE_SPIN") == "1":
        # hipDeviceScheduleSpin (1) before anything creates the context
        rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1))
        print("hipSetDeviceFlags rc", rc, file=sys.stderr)
    import torch
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda", 0)
    ring = 400
    env, st, acts = bench._env_and_actions(dev, envs, 0, 0, 2000, ring)
    sp = ctypes.c_void_p(st.cuda_stream)
    done = torch.empty(envs, dtype=torch.uint8, device=dev)
    ap, dp = ctypes.c_void_p(acts.data_ptr()), ctypes.c_void_p(done.data_ptr())
    fn, h, lim, rp = env._L.sk_env_step_multi, env._h, env.tick_limit, int(env.random_positions)
    slab = 0

    def run():
        nonlocal slab
        rc = fn(h, ap, ring, slab, k, dp, None, 0, lim, 1, rp, sp)
        assert rc == 0, rc
        slab = (slab + k) % ring

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    e1.record(st)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    rows = {}

    def add(name, v):
        rows.setdefault(name, []).append(v)

    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        run()
        e1.record(st)
        torch.cuda.synchronize()
        add("wall", (time.perf_counter() - t0) * 1e6)
        add("event", e0.elapsed_time(e1) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        run()
        e1.record(st)
        while not e1.query():
            pass
        torch.cuda.synchronize()
        add("wall_poll", (time.perf_counter() - t0) * 1e6)
        add("event_poll", e0.elapsed_time(e1) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        e1.record(st)
        torch.cuda.synchronize()
        add("empty", (time.perf_counter() - t0) * 1e6)
    out = {name: round(statistics.median(v), 2) for name, v in rows.items()}
    out.update(k=k, envs=envs, unit="us per region (median)")
    env.close()
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--reps", type=int, default=40)
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--only", default="")
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        print(json.dumps(child(a.k, a.reps, a.envs)), flush=True)
        return
    names = [s for s in a.only.split(",") if s] or list(SETTINGS)
    for name in names:
        env = dict(os.environ, **SETTINGS[name])
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--k", str(a.k), "--reps", str(a.reps),
               "--envs", str(a.envs)]
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
            d = json.loads(line) if line else {"error": r.stderr[-400:], "rc": r.returncode}
        except subprocess.TimeoutExpired:
            d = {"error": "timeout"}
        d["setting"] = name
        print(json.dumps(d), flush=True)
        if "error" in d:
            break


if __name__ == "__main__":
    main()
