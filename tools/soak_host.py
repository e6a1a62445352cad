"""Randomized soak of the table-function host on the GPU box (robustness;
a shortened seeded form runs in the GPU suite, tests/test_soak_gpu.py).

For a wall-clock budget it runs tools/host_e2e on seeded random query shapes:
table size, executor threads, batch_size (down to a few rows: many slots and
ring wraps), row chunks, DuckDB vectors or Arrow columns, 0 / 1 / 2 / 16 label keys, fixed or
ragged output lists, 1 / 3 / 8 logical GPUs on the one card, streaming feeds or
per-slot launches, the streaming slot count, plain or non-temporal slot copies,
the spend-key fold on or off, streaming kernels that leave after 1-3 ms idle
(relaunched by the next publish), output_count 1..13 and label negation (the
planted values, index 0 and added labels, match under every variant).  Every query must emit exactly the planted rows
(host_e2e's own check), and each run's 512-row sample is recomputed by the C
oracle (oracle.check_planted_sample, checker use of oracle/).  Prints one line
per run and a JSON summary; exit 1 on the first failure.

  python tools/soak_host.py --minutes 8 --seed 1 --out gpurun_out/soak.jsonl

tests/test_soak_gpu.py runs a seeded one-minute form in the GPU suite
(streaming feeds with 4 slots, the shape that lost matches to stale cached
slots in round 5).
"""
import argparse
import json
import os
import random
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shape(rng):
    rows = rng.choice([1, 777, 2048, 2049, 65536, 300001, 1_000_000, 2_500_000])
    labels = rng.choice([0, 0, 1, 2, 16])
    return dict(
        rows=rows,
        threads=rng.choice([1, 2, 3, 8, 16, 32]),
        batch=rng.choice([1, 7, 2048, 5000, 65536, 300000]),
        input=rng.choice(["rows", "columns", "vectors"]),
        labels=labels,
        outputs=rng.choice([["--outputs", "1"], ["--outputs", "2"], ["--outputs", "8"], ["--outputs-max", "15"]]),
        device_map=rng.choice(["0", "0", "0,0,0", ",".join(["0"] * 8)]),
        mode=rng.choice(["", "stream", "launch"]),  # "": streaming for one feed per device, else per-slot
        slots=rng.choice(["", "", "4", "48"]),
        nt=rng.choice(["", "0"]),
        fold=rng.choice(["", "0"]),
        reps=rng.choice([1, 2]),
        idle_ms=rng.choice(["", "", "1", "3"]),  # streaming kernels leave when idle this long: many relaunches
        output_count=rng.choice([1, 1, 1, 2, 6, 7, 13]),  # protocol variants: > 6 = WIDE
        label_negation=rng.choice([False, False, False, True]),
    )


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=8.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--timeout", type=int, default=240, help="seconds per run")
    ap.add_argument("--mode", default=None, choices=["", "stream", "launch"],
                    help="fix the host mode for every run (default: random)")
    ap.add_argument("--slots", default=None, help="fix CUDASP_TF_STREAM_SLOTS for every run (default: random)")
    ap.add_argument("--max-rows", type=int, default=0, help="cap every run's table (0 = no cap)")
    a = ap.parse_args()
    import bench
    from oracle import oracle
    exe = os.path.join(ROOT, "tools", "host_e2e")
    rng = random.Random(a.seed)
    t_end = time.time() + 60 * a.minutes
    runs, queries, rows_total, sample_rows = 0, 0, 0, 0
    out = open(a.out, "w") if a.out else None
    while time.time() < t_end:
        sh = shape(rng)
        if a.mode is not None:
            sh["mode"] = a.mode
        if a.slots is not None:
            sh["slots"] = a.slots
        if a.max_rows:
            sh["rows"] = min(sh["rows"], a.max_rows)
        # tiny batches on big tables take many slot cycles, K indices K x stage B:
        # keep a run bounded
        if sh["batch"] < 2048 and sh["rows"] > 65536:
            sh["rows"] = 65536
        if sh["output_count"] > 2 and sh["rows"] > 300001:
            sh["rows"] = 300001
        env = dict(os.environ, CUDASP_TF_DEVICE_MAP=sh["device_map"])
        if sh["mode"] == "stream" and "," in sh["device_map"]:
            env["GPU_MAX_HW_QUEUES"] = "16"  # a hardware queue per feed's persistent kernel (as the 8-feed test)
        for k, v in (("CUDASP_TF_MODE", sh["mode"]), ("CUDASP_TF_STREAM_SLOTS", sh["slots"]),
                     ("CUDASP_TF_NT", sh["nt"]), ("CUDASP_FB_FOLD", sh["fold"]),
                     ("CUDASP_STREAM_IDLE_MS", sh["idle_ms"])):
            env.pop(k, None)
            if v:
                env[k] = v
        smp = tempfile.NamedTemporaryFile(prefix="soak_sample_", suffix=".json", delete=False)
        smp.close()
        cmd = [exe, "--rows", str(sh["rows"]), "--threads", str(sh["threads"]), "--batch", str(sh["batch"]),
               "--input", sh["input"], "--labels", str(sh["labels"]), "--reps", str(sh["reps"]),
               "--plant-sample", smp.name, "--output-count", str(sh["output_count"])] + sh["outputs"]
        if sh["label_negation"]:
            cmd.append("--label-negation")
        lf = None
        if sh["labels"]:
            lf = tempfile.NamedTemporaryFile(prefix="soak_labels_", suffix=".bin", delete=False)
            lf.write(b"".join(bench.label_keys(sh["labels"])))
            lf.close()
            cmd += ["--labels-file", lf.name]
        t0 = time.time()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, env=env)
        except subprocess.TimeoutExpired:
            print(json.dumps(dict(shape=sh, error="timed out")), flush=True)
            sys.exit(1)
        finally:
            if lf is not None:
                os.unlink(lf.name)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
        res = json.loads(line) if line.startswith("{") else {}
        ok = r.returncode == 0 and res.get("emitted_equal_planted") is True
        chk = {}
        if ok:
            with open(smp.name) as f:
                chk = oracle.check_planted_sample(json.load(f), threads=8)
            ok = chk["equal"] == chk["rows"]
        os.unlink(smp.name)
        runs += 1
        queries += 1 + sh["reps"]
        rows_total += sh["rows"] * (1 + sh["reps"])
        sample_rows += chk.get("rows", 0)
        rec = dict(run=runs, ok=ok, seconds=round(time.time() - t0, 2), shape=sh,
                   tx_per_s=res.get("tx_per_s"), launches=res.get("launches"),
                   streaming_feeds=res.get("streaming_feeds"), oracle_sample=[chk.get("equal"), chk.get("rows")])
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
            out.flush()
        if not ok:
            print(json.dumps(dict(failed=sh, exit=r.returncode, stderr=r.stderr[-2000:], mismatches=chk.get("mismatches"))),
                  flush=True)
            sys.exit(1)
    print(json.dumps(dict(soak="ok", seed=a.seed, minutes=a.minutes, runs=runs, queries=queries, rows=rows_total,
                          oracle_sample_rows=sample_rows)), flush=True)


if __name__ == "__main__":
    main()
