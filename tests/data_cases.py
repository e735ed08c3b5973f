"""A small on-disk crater dataset in the reference's layout, written on the fly for the data-path
tests (altitude*/longitude*/truth/detections.csv + images next to truth/)."""
from __future__ import annotations

from pathlib import Path

import numpy as np


def make_dataset(root: Path, seed: int = 0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    specs = [("altitude01/longitude10", [("a.png", (480, 640), "L"), ("b.png", (700, 517), "L"),
                                         ("c.png", (640, 640), "L")]),
             ("altitude02/longitude03", [("d.png", (300, 401), "RGB"), ("e.png", (1024, 1024), "L")])]
    rows_all = {}
    for sub, imgs in specs:
        d = root / sub
        (d / "truth").mkdir(parents=True, exist_ok=True)
        rows = []
        for name, (h, w), mode in imgs:
            if mode == "L":
                a = rng.integers(0, 256, (h, w), dtype=np.uint8)
            else:
                a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
            Image.fromarray(a, mode).save(d / name)
            for k in range(int(rng.integers(1, 6))):
                cls = [0, 1, 2, 3, 4, -1, None][int(rng.integers(0, 7))]
                rows.append({"inputImage": name, "ellipseCenterX(px)": float(rng.uniform(-5, w + 5)),
                             "ellipseCenterY(px)": float(rng.uniform(-5, h + 5)),
                             "ellipseSemimajor(px)": float(rng.uniform(1, w / 3)),
                             "ellipseSemiminor(px)": float(rng.uniform(0.5, h / 3)),
                             "crater_classification": cls})
        # a row whose image is missing is skipped by the loader
        rows.append({"inputImage": "missing.png", "ellipseCenterX(px)": 1.0, "ellipseCenterY(px)": 1.0,
                     "ellipseSemimajor(px)": 1.0, "ellipseSemiminor(px)": 1.0, "crater_classification": 1})
        import pandas as pd
        pd.DataFrame(rows).to_csv(d / "truth" / "detections.csv", index=False)
        rows_all[sub] = rows
    return rows_all
