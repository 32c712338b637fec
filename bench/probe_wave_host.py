"""Host-side anatomy of the gap between two bench waves (the time the GPU waits on Python).

Runs bench.py's headline workload (same flags) with timestamps on: the engine completing the
last sequence of a wave, the client's first / last submission of the next wave, the engine thread
draining them, the prefill step's start and end, and the first decode window's launch. Prints one
JSON line per wave boundary and a median summary.

    python bench/probe_wave_host.py --steps 4 --warmup 1
"""

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from src.engine import llm_engine, model_runner  # noqa: E402
from src.engine import async_engine  # noqa: E402

EV = []


def mark(name):
    EV.append((time.perf_counter(), name))


def wrap(cls, meth, before=None, after=None):
    f = getattr(cls, meth)

    def g(self, *a, **k):
        if before:
            mark(before)
        r = f(self, *a, **k)
        if after:
            mark(after)
        return r

    setattr(cls, meth, g)


wrap(async_engine.AsyncLLMEngine, "submit", before="submit")
wrap(async_engine.AsyncLLMEngine, "_drain_submissions", after="drained")
wrap(llm_engine.LLMEngine, "_complete", after="complete")
wrap(llm_engine.LLMEngine, "add_request", after="add_request")
wrap(model_runner.ModelRunner, "prefill", before="prefill_start", after="prefill_end")
wrap(model_runner.ModelRunner, "decode_multi", before="decode_multi")
wrap(llm_engine.LLMEngine, "step", before="step")


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    bench.main()
    ev = sorted(EV)
    # wave boundaries: a prefill_start preceded by completes
    out = []
    for i, (t, n) in enumerate(ev):
        if n != "prefill_start":
            continue
        prev = [x for x in ev[:i] if x[1] == "complete"]
        if not prev:
            continue
        t_done = prev[-1][0]
        sub = [x[0] for x in ev[:i] if x[1] == "submit" and x[0] > t_done]
        drn = [x[0] for x in ev[:i] if x[1] == "drained" and x[0] > t_done]
        steps = [x[0] for x in ev[:i] if x[1] == "step" and x[0] > t_done]
        pend = next(x[0] for x in ev[i:] if x[1] == "prefill_end")
        dm = next((x[0] for x in ev[i:] if x[1] == "decode_multi"), None)
        if not sub:
            continue
        out.append({"done_to_first_submit_ms": 1e3 * (sub[0] - t_done),
                    "submit_span_ms": 1e3 * (sub[-1] - sub[0]),
                    "last_submit_to_drained_ms": 1e3 * (max(drn) - sub[-1]) if drn else None,
                    "engine_steps_in_gap": len(steps),
                    "last_submit_to_prefill_ms": 1e3 * (t - sub[-1]),
                    "done_to_prefill_ms": 1e3 * (t - t_done),
                    "prefill_ms": 1e3 * (pend - t),
                    "prefill_end_to_decode_ms": 1e3 * (dm - pend) if dm else None})
    for o in out:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in o.items()}))
    if out:
        keys = [k for k in out[0] if isinstance(out[0][k], (int, float))]
        print(json.dumps({"median": {k: round(statistics.median(o[k] for o in out if o[k] is not None), 3)
                                     for k in keys}}))


if __name__ == "__main__":
    main()
