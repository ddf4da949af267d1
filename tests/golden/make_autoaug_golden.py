"""Writes tests/golden/autoaug_policies_ref.json: the AutoAugment sub-policy tables the reference
itself holds (/root/reference/utils/augment.py:24-163, ImageNetPolicy / CIFAR10Policy /
SVHNPolicy), parsed as TEXT (nothing from the reference is imported or executed).

Each SubPolicy(p1, "op1", mag_idx1, p2, "op2", mag_idx2, fill) becomes
[[Op1, p1, bin1], [Op2, p2, bin2]] with the op renamed to torchvision's AutoAugment spelling
and bin = None for the ops torchvision applies without a magnitude (Invert, AutoContrast,
Equalize) — the form of lcclip.transforms.AUTOAUG_POLICIES, so the test compares the two
directly. The reference trains with torchvision's AutoAugment (methods/_trainer.py:217-228);
these tables are the same published policies, held in the reference's own tree.

Run from the repo root in a container that has /root/reference:
    python tests/golden/make_autoaug_golden.py
"""
import json
import os
import re

SRC = "/root/reference/utils/augment.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "autoaug_policies_ref.json")
NAMES = {"shearX": "ShearX", "shearY": "ShearY", "translateX": "TranslateX",
         "translateY": "TranslateY", "rotate": "Rotate", "color": "Color",
         "posterize": "Posterize", "solarize": "Solarize", "contrast": "Contrast",
         "sharpness": "Sharpness", "brightness": "Brightness", "autocontrast": "AutoContrast",
         "equalize": "Equalize", "invert": "Invert"}
NO_MAG = {"AutoContrast", "Equalize", "Invert"}
CLASSES = {"ImageNetPolicy": "imagenet", "CIFAR10Policy": "cifar10", "SVHNPolicy": "svhn"}
SUB = re.compile(r'SubPolicy\(\s*([0-9.]+)\s*,\s*"(\w+)"\s*,\s*(\d+)\s*,\s*([0-9.]+)\s*,'
                 r'\s*"(\w+)"\s*,\s*(\d+)\s*,')


def parse(text):
    out = {}
    # split the file at each policy class header; the SubPolicy lines up to the next class belong to it
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^class (\w+)\(", text, re.M)]
    for i, (pos, cls) in enumerate(heads):
        if cls not in CLASSES:
            continue
        end = heads[i + 1][0] if i + 1 < len(heads) else len(text)
        rows = []
        for m in SUB.finditer(text[pos:end]):
            p1, o1, b1, p2, o2, b2 = m.groups()
            ent = []
            for p, op, b in ((p1, o1, b1), (p2, o2, b2)):
                name = NAMES[op]
                ent.append([name, float(p), None if name in NO_MAG else int(b)])
            rows.append(ent)
        out[CLASSES[cls]] = rows
    return out


if __name__ == "__main__":
    tables = parse(open(SRC).read())
    assert sorted(tables) == ["cifar10", "imagenet", "svhn"], sorted(tables)
    json.dump({"source": "reference utils/augment.py:24-163 (parsed as text)", "policies": tables},
              open(OUT, "w"), indent=1)
    print({k: len(v) for k, v in tables.items()}, "->", OUT)
