import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f)); print(f, d["value"], {k: round(v["us"], 2) for k, v in d["kernels"].items()})
