"""Compact view of dgrad_epi_probe JSON lines: shape variant loop best_cfg best_us TB/s."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        r = json.loads(line)
        print(r["shape"][:9], r["variant"], r.get("loop", 1), r["best_cfg"], r["best_us"], r["TBps"])
