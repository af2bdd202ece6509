"""Host enqueue rate against GPU rate of the learner's tick graphs: is the
graph-replayed learner tick host-bound?  Config 3's shape (bench.learner_rate:
4,096 games, action noise, fp32, batch 256) by default.  For each
ticks-per-graph value: the host time of each TickGraph replay call, the HIP
event time of every replay (events on the graph's stream between replays),
and the whole region's events per tick.  One JSON line per value.  The
default loop replays on the capture stream with events between replays;
--via-run times TickGraph.run(n); --mode times run()'s body inline with its
stream waits switched on and off (the bisection behind run()'s form).

    python tools/graph_host_rate.py [--envs 4096] [--tpg 2,10,40] [--ticks 400]"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--tpg", default="2,10,40")
    p.add_argument("--ticks", type=int, default=400)
    p.add_argument("--exploration", default="action_noise")
    p.add_argument("--precision", default="fp32")
    p.add_argument("--warm", type=int, default=20, help="warm-up ticks")
    p.add_argument("--via-run", action="store_true", help="time one TickGraph.run(n) (bench.learner_rate's way)")
    p.add_argument("--mode", default="", help="time run()'s body inline with pieces: 'ws' (stream waits), 'pre' / 'post' (one of them), 'query' (the first wait only if the current stream is busy), 'sync'")
    a = p.parse_args()
    from skillshot_learning_amd.learner import SkillshotLearner
    for tpg in [int(x) for x in a.tpg.split(",")]:
        L = SkillshotLearner(n_envs=a.envs, seed=0, exploration=a.exploration, tick_limit=2000,
                             replay_capacity=1 << 20, gamma=0.99, tau=0.005, precision=a.precision)
        tg = L.tick_graph(batch=256, updates_per_tick=1, ticks_per_graph=tpg)
        tg.run(max(1, a.warm // tpg))
        torch.cuda.synchronize()
        n = max(1, a.ticks // tpg)
        if a.via_run or a.mode:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
            st = tg.stream
            if "cur" in a.mode or a.via_run:  # TickGraph.run replays on the caller's stream
                st = torch.cuda.current_stream(L.device)
            e0.record(st)
            h0 = time.perf_counter()
            if a.via_run:
                tg.run(n)
            else:  # TickGraph.run's body, pieces switched by --mode
                cur = torch.cuda.current_stream(L.device)
                if "ws" in a.mode or "pre" in a.mode:
                    st.wait_stream(cur)
                if "query" in a.mode and not cur.query():
                    st.wait_stream(cur)
                if "cur" in a.mode:  # replay on the current stream itself: no cross-stream waits
                    st = cur
                with torch.cuda.stream(st):
                    if "sync" in a.mode:
                        L.game_environment.sync_step_counter(ctypes.c_void_p(st.cuda_stream))
                    for i in range(n):
                        kind, g = tg._phases[tg._phase]
                        g.replay()
                        if "ev" in a.mode:
                            evs[i].record(st)
                        tg._phase = (tg._phase + tg.ticks) % 2
                if "ws" in a.mode or "post" in a.mode or "query" in a.mode:
                    cur.wait_stream(st)
                if "hsync" in a.mode:
                    st.synchronize()
            h1 = time.perf_counter()
            e1.record(st)
            torch.cuda.synchronize()
            print(json.dumps(dict(envs=a.envs, ticks_per_graph=tpg, warm=a.warm, via_run=a.via_run, mode=a.mode,
                                  host_us=(h1 - h0) * 1e6, gpu_us_per_tick_mean=e0.elapsed_time(e1) * 1e3 / (n * tpg),
                                  per_replay_us=[round(evs[i - 1].elapsed_time(evs[i]) * 1e3, 1) for i in range(1, n)]
                                  if "ev" in a.mode else None,
                                  last_to_e1_us=evs[-1].elapsed_time(e1) * 1e3 if "ev" in a.mode else None)),
                  flush=True)
            del tg, L
            torch.cuda.empty_cache()
            continue
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        host = []
        # TickGraph.run's replay loop with an event after every replay (the
        # host mirrors it also advances are not needed: the learner is dropped)
        st = tg.stream
        with torch.cuda.stream(st):
            L.game_environment.sync_step_counter(ctypes.c_void_p(st.cuda_stream))
            ev[0].record(st)
            t0 = time.perf_counter()
            for i in range(n):
                kind, g = tg._phases[tg._phase]
                assert kind == "graph"
                h0 = time.perf_counter()
                g.replay()
                host.append(time.perf_counter() - h0)
                ev[i + 1].record(st)
                tg._phase = (tg._phase + tg.ticks) % 2
            t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        gpu = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)]  # us per replay
        out = dict(envs=a.envs, ticks_per_graph=tpg, replays=n, warm=a.warm, per_replay_us=[round(x, 1) for x in gpu],
                   host_us_per_replay_median=statistics.median(host) * 1e6,
                   host_us_per_tick=statistics.median(host) * 1e6 / tpg,
                   gpu_us_per_replay_median=statistics.median(gpu), gpu_us_per_tick_median=statistics.median(gpu) / tpg,
                   gpu_us_per_tick_mean=sum(gpu) / n / tpg,
                   gpu_us_per_tick_p90=sorted(gpu)[int(0.9 * n)] / tpg,
                   enqueue_s=t_enq, wall_s=t_all, wall_us_per_tick=t_all * 1e6 / (n * tpg))
        print(json.dumps(out), flush=True)
        del tg, L
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
