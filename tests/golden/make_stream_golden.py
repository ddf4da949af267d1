"""Extract the Si-Blurry known answer from the reference's own run log (nohup.out:1, 10-21):
config {'dataset': 'cifar100', 'n_tasks': 10, 'n': 100, 'm': 0, 'rnd_NM': False, 'rnd_seed': 0}
and the logged per-task disjoint class lists / task sizes. That run used the sampler's
random class order (torch.randperm under the seed; HEAD switched to torch.arange, see
utils/online_sampler.py:57-58), so the fixture pins class_order='random'.
Runs here only (reads /root/reference as text); the JSON it writes is the committed fixture."""
import ast
import json
import os
import re

SRC = "/root/reference/nohup.out"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "siblurry_cifar100_seed0.json")

lines = open(SRC).read().splitlines()
cfg = ast.literal_eval(lines[0].split("| ", 1)[1])
disj = blur = None
sizes = []
for ln in lines:
    if "| disjoint classes: " in ln and disj is None:
        disj = ast.literal_eval(ln.split("disjoint classes: ", 1)[1])
    elif "| blurry classes: " in ln and blur is None:
        blur = ast.literal_eval(ln.split("blurry classes: ", 1)[1])
    m = re.search(r"task (\d+): disjoint (\d+), blurry (\d+)", ln)
    if m:
        sizes.append([int(m.group(2)), int(m.group(3))])
fixture = {
    "source": "qcNPU/LifeLong-CLIP nohup.out lines 1, 10-21",
    "config": {k: cfg[k] for k in ("dataset", "n_tasks", "n", "m", "rnd_NM", "rnd_seed", "memory_size")},
    "disjoint_classes": disj,
    "blurry_classes": blur,
    "task_sizes_disjoint_blurry": sizes[:cfg["n_tasks"]],
}
json.dump(fixture, open(OUT, "w"), indent=1)
print(OUT, {k: (v if k != "disjoint_classes" else "...") for k, v in fixture.items()})
