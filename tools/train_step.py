"""Config-3 training step alone (bench.train_bench): for rocprofv3 kernel traces of the train
step without the forward bench around it.  python tools/train_step.py [--steps K --warmup W]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--clips", type=int, default=8)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--serial-teacher", dest="concurrent_teacher", action="store_false")
    ap.add_argument("--concurrent-groups", dest="concurrent_groups", action="store_true")
    ap.add_argument("--no-teacher-train", action="store_true",
                    help="skip the teacher-train-mode leg (the trace then ends with the timed steps)")
    ap.add_argument("--host-time", action="store_true",
                    help="also report the host-side enqueue time of each step (no sync inside the step)")
    a = ap.parse_args()
    if a.host_time:
        import time
        from dsvt import trainer as _tr
        _orig = _tr.DINOTrainer.step
        host = []

        def _timed(self, *args, **kw):
            t0 = time.perf_counter()
            r = _orig(self, *args, **kw)
            host.append(time.perf_counter() - t0)
            return r
        _tr.DINOTrainer.step = _timed
    torch.cuda.set_device(0)
    print(json.dumps(bench.train_bench(a, torch.device("cuda", 0), 0, 1, a.steps, a.warmup)), flush=True)
    if a.host_time:
        print(json.dumps({"host_enqueue_ms_per_step": [round(h * 1e3, 2) for h in host]}), flush=True)
