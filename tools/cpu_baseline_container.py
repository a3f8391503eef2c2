#!/usr/bin/env python3
"""Time bench.py's single-core CPU baselines (the oracle restatements) in the build container,
the machine class the survey's reference rates were measured on (an 8-core
Xeon VM), and write profiles/<out>.json.  bench.py quotes it as `validated_rate`: the same
loop on the same kind of host as the survey, against the survey's compute-only rates."""
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r05_cpu_baseline_container.json")
    l8 = bench.cpu_baseline_lyon8(128, 128, 20000)
    b22 = bench.cpu_baseline_bates22(128, 200)
    cpu = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    res = {
        "host": {"cpu": cpu, "cpus": os.cpu_count(), "python": platform.python_version()},
        "measured": time.strftime("%Y-%m-%d"),
        "lyon8": {"value": l8["value"], "survey_compute_only": 736.0,
                  "ratio_to_survey": l8["value"] / 736.0, "sample": l8["sample"]},
        "bates22": {"value": b22["value"], "survey_compute_only": 17.0,
                    "ratio_to_survey": b22["value"] / 17.0, "sample": b22["sample"]},
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
