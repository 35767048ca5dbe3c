import json, os, sys
sys.path.insert(0, os.getcwd())
import bench, lpcnet_amd as L
blob = L.synthetic_model(1, 0)
for B in (1024, 1):
    print(B, json.dumps(bench.latency(L, blob, B, 0.0), indent=1))
