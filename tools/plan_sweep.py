"""Sweep fast-kernel plans (ME_PLAN="K,tb,cpp,threads") on one workload and
print kernel time per plan, next to the planner's own choice ("auto").
usage: plan_sweep.py --width W --height H --blk B --span S --cost sad|ssd"""
import argparse
import itertools
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--blk", type=int, default=16)
    ap.add_argument("--span", type=int, default=32)
    ap.add_argument("--cost", default="sad")
    ap.add_argument("--K", default="13,11,8")
    ap.add_argument("--tb", default="1,2,3,4,5,6")
    ap.add_argument("--cpp", default="0")
    ap.add_argument("--threads", default="256")
    ap.add_argument("--fold", default="-1")
    ap.add_argument("--plans", default="", help="explicit 'K,tb,cpp,thr,fold;...' (overrides the grid)")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rows", default="", help="block rows r0:r1 (one row stripe)")
    a = ap.parse_args()
    plans = ["auto"] + [f"{k},{t},{c},{n},{f}" for k, t, c, n, f in itertools.product(
        a.K.split(","), a.tb.split(","), a.cpp.split(","), a.threads.split(","),
        a.fold.split(","))]
    if a.plans:
        plans = ["auto"] + a.plans.split(";")
    for plan in plans:
        env = dict(os.environ, ME_HIP_LIB="libme_hip_tune.so")  # ME_PLAN: tuning build only
        if plan != "auto":
            env["ME_PLAN"] = plan
        r = subprocess.run([sys.executable, os.path.join(HERE, "size_sweep.py"), "--cost", a.cost,
                            "--blk", str(a.blk), "--span", str(a.span), "--width", str(a.width),
                            "--heights", str(a.height), "--iters", str(a.iters)] +
                           (["--rows", a.rows] if a.rows else []),
                           env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not line:
            print(json.dumps({"plan": plan, "error": (r.stderr or r.stdout)[-300:]}), flush=True)
            continue
        d = json.loads(line[-1])
        print(json.dumps({"plan": plan, "ms": round(d["ms"], 5), "cand_per_s": d["cand_per_s"]}),
              flush=True)


if __name__ == "__main__":
    main()
