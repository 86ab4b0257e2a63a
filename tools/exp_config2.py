"""Config 2 (BASELINE configs[1]: 4,096 envs, b747_model_step) alone: bench.py's config2_rates line, ROUNDS times.
Run on the GPU box: python tools/exp_config2.py [rounds]   (B747_LIB_PATH selects an A/B build)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    d = bench.config2_rates(dev)
    print(json.dumps({"lib": os.path.basename(os.environ.get("B747_LIB_PATH", "libb747.so")),
                      "step_us": d["step"]["us_per_step"], "multi_step_us": d["multi_step"]["us_per_step"],
                      "step_rate": d["step"]["value"], "multi_rate": d["multi_step"]["value"]}), flush=True)
