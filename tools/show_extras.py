"""Print the headline value and the config-3/5 phase times of a bench.py JSON line.
usage: python tools/show_extras.py bench.json"""
import json
import sys

d = json.load(open(sys.argv[1]))
print("value %.1f G" % (d["value"] / 1e9))
for k in ("a3c_config3", "a3c_config3_reference", "dqn_config5"):
    e = d.get("extras", {}).get(k, {})
    print(k, {x: round(e[x], 3) for x in ("rollout_ms", "update_ms", "act_ms") if e.get(x) is not None})
