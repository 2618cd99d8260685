"""print 'tag value ms_per_step host_issue' from a bench.py log"""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith('{"metric'):
        d = json.loads(line)
        print(sys.argv[2] if len(sys.argv) > 2 else "", d["value"], d["ms_per_step"], "host issue",
              d.get("host_issue_ms_per_step"), "grace", d.get("grace_ms_per_step"), flush=True)
