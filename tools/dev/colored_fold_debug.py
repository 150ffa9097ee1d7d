"""Dev probe: BatchAugmenter output with and without the colored fold, twice each."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from test_augment import _clips, _bank
from heybuddy.dataset.augmented import BatchAugmenter
noises, irs = _bank(seed=42)
xb = torch.from_numpy(_clips(300, seed=44)).float().cuda()
outs = {}
for tag, fold in (("fold1", "1"), ("nofold1", "0"), ("fold2", "1"), ("nofold2", "0")):
    os.environ["HBK_AUG_COLORED_FOLD"] = fold
    np.random.seed(9)
    torch.manual_seed(9)
    aug = BatchAugmenter([torch.from_numpy(v).float() for v in noises], [torch.from_numpy(v).float() for v in irs],
                         device=0, batch_size=128, colored_noise_prob=1.0, tanh_distortion_prob=0.0,
                         seven_band_prob=0.0, band_stop_prob=0.0, pitch_shift_prob=0.0)
    pr = aug.prepare(300)
    print(tag, "colored:", None if pr["colored"] is None else (pr["colored"][0][:3].tolist(), pr["colored"][1][::128].tolist(), pr["colored"][2]),
          "gain", None if pr["gain"] is None else pr["gain"][::128].tolist())
    outs[tag] = aug(xb, prepared=pr).clone()
for a, b in (("fold1", "fold2"), ("nofold1", "nofold2"), ("fold1", "nofold1")):
    d = (outs[a] - outs[b]).abs()
    rows = torch.nonzero(d.amax(1) > 0).reshape(-1).tolist()
    print(a, b, "max", float(d.max()), "rows differing", len(rows), rows[:10])
