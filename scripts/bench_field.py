"""Prints one field of the bench.py JSON line found in a log: bench_field.py LOG a.b.c"""
import json
import sys

val = None
for line in open(sys.argv[1], errors="replace"):
    line = line.strip()
    if line.startswith("{") and '"metric"' in line:
        val = json.loads(line)
for k in sys.argv[2].split("."):
    val = val[k]
print(val)
