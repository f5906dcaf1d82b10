"""Episode-end example pipeline: columnar training examples instead of pickled tuples.

The reference assembles one tuple per example (Coach.py:89-98)

    (board int8[R,7], pi float[409], winner float[n], scdiff int[n], valids bool[409],
     surprise float[n])

and stores each one `zlib.compress(pickle.dumps(x))` (Coach.py:100), the iteration history
pickled whole (`saveTrainExamples`, Coach.py:167-173); training decompresses per sample
(`GenericNNetWrapper.pick_examples`, :326-331) and weighs samples by surprise
(`compute_surprise_weights`, :333-340).

Here an `ExampleSet` keeps the same six fields as columns (device or host tensors, straight
from `SelfPlay.drain()` + `symmetries`), valids bit-packed as the engine's 7 x u64 mask
words. On disk it is a plain `.npz` (numpy arrays only, read back with allow_pickle=False:
nothing is unpickled), optionally deflate-compressed like the reference's zlib level.
`ExampleHistory` is the trainExamplesHistory window (numItersHistory iterations) saved as
one `checkpoint.examples.npz`.
"""
import os

import numpy as np
import torch

from .env import ACTIONS, MASK_WORDS, pack_mask, unpack_mask

FIELDS = ("board", "pi", "winner", "scdiff", "valids", "surprise")
_FORMAT = 1


class ExampleSet:
    """Columnar examples; `valids` is packed [E, 7] int64 (engine mask words)."""

    def __init__(self, board, pi, winner, scdiff, valids, surprise):
        self.board, self.pi, self.winner = board, pi, winner
        self.scdiff, self.valids, self.surprise = scdiff, valids, surprise
        E = board.shape[0]
        for k in FIELDS:
            t = getattr(self, k)
            if t.shape[0] != E:
                raise ValueError(f"field {k}: {t.shape[0]} rows, board has {E}")
        if valids.ndim != 2 or valids.shape[1] != MASK_WORDS:
            raise ValueError(f"valids must be packed [E, {MASK_WORDS}] mask words")

    # ------------------------------------------------------------ construction
    @classmethod
    def from_drain(cls, ex):
        """From SelfPlay.drain() / coach.expand_symmetries output (dict of tensors)."""
        return cls(*(ex[k] for k in FIELDS))

    @classmethod
    def from_tuples(cls, examples):
        """From the reference's list of (board, pi, winner, scdiff, valids, surprise)."""
        if not examples:
            raise ValueError("no examples")
        cols = list(zip(*examples))
        board = torch.from_numpy(np.stack([np.asarray(b, np.int8) for b in cols[0]]))
        pi = torch.from_numpy(np.stack([np.asarray(p, np.float32) for p in cols[1]]))
        winner = torch.from_numpy(np.stack([np.asarray(w, np.float32) for w in cols[2]]))
        scdiff = torch.from_numpy(np.stack([np.asarray(s, np.int32) for s in cols[3]]))
        valids = pack_mask(torch.from_numpy(np.stack([np.asarray(v, bool) for v in cols[4]])))
        surprise = torch.from_numpy(np.stack([np.asarray(s, np.float32) for s in cols[5]]))
        return cls(board, pi, winner, scdiff, valids, surprise)

    @classmethod
    def cat(cls, sets):
        sets = [s for s in sets if len(s)]
        if not sets:
            raise ValueError("no examples")
        dev = sets[0].board.device
        return cls(*(torch.cat([getattr(s, k).to(dev) for s in sets]) for k in FIELDS))

    def __len__(self):
        return int(self.board.shape[0])

    def to(self, device):
        return ExampleSet(*(getattr(self, k).to(device) for k in FIELDS))

    def to_tuples(self):
        """The reference's per-example tuples (Coach.py:91-98), valids unpacked to bool."""
        h = self.to("cpu")
        valids = unpack_mask(h.valids).numpy()
        cols = [h.board.numpy(), h.pi.numpy(), h.winner.numpy(), h.scdiff.numpy(), valids,
                h.surprise.numpy()]
        return [tuple(c[i] for c in cols) for i in range(len(self))]

    # ------------------------------------------------------------ training-side access
    def pick_examples(self, sample_ids):
        """GenericNNetWrapper.pick_examples (:326-331): the six columns of the picked
        samples (a tuple of per-field batches instead of a tuple of tuples)."""
        idx = torch.as_tensor(np.asarray(sample_ids, dtype=np.int64), device=self.board.device)
        out = [getattr(self, k).index_select(0, idx) for k in FIELDS]
        out[4] = unpack_mask(out[4])
        return tuple(out)

    def compute_surprise_weights(self):
        """GenericNNetWrapper.compute_surprise_weights (:333-340), same formula and shape:
        x[-1] is the example's surprise vector [n]; weights = s / s.sum() + 1/len,
        renormalised by the grand total (NumPy's .sum() over every element)."""
        s = self.surprise.detach().cpu().numpy()
        w = s / s.sum() + 1. / len(s)
        return w / w.sum()

    # ------------------------------------------------------------ storage
    def arrays(self):
        h = self.to("cpu")
        return {k: getattr(h, k).numpy() for k in FIELDS}

    def save(self, path, compress=True):
        """Write a .npz (numpy arrays only; `compress` = deflate, the reference's zlib)."""
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        arrs = dict(self.arrays(), format=np.int32(_FORMAT), actions=np.int32(ACTIONS))
        (np.savez_compressed if compress else np.savez)(path, **arrs)

    @classmethod
    def load(cls, path, device="cpu"):
        with np.load(path, allow_pickle=False) as z:
            if int(z["format"]) != _FORMAT or int(z["actions"]) != ACTIONS:
                raise ValueError(f"{path}: unsupported example file (format {int(z['format'])})")
            return cls(*(torch.from_numpy(z[k]).to(device) for k in FIELDS))


class ExampleHistory:
    """Coach.trainExamplesHistory: one ExampleSet per iteration, at most `max_iters`
    (args.numItersHistory, Coach.py:134-135), saved/loaded as checkpoint.examples.npz
    (saveTrainExamples / loadTrainExamples, Coach.py:167-190)."""

    FILE = "checkpoint.examples.npz"

    def __init__(self, max_iters=None):
        self.max_iters = max_iters
        self.iters = []

    def append(self, exset):
        self.iters.append(exset)
        if self.max_iters is not None and len(self.iters) > self.max_iters:
            self.iters.pop(0)

    def __len__(self):
        return sum(len(s) for s in self.iters)

    def merged(self):
        return ExampleSet.cat(self.iters)

    def save(self, folder, compress=True):
        os.makedirs(folder, exist_ok=True)
        sizes = np.array([len(s) for s in self.iters], np.int64)
        merged = self.merged().arrays() if len(sizes) and sizes.sum() else {}
        path = os.path.join(folder, self.FILE)
        (np.savez_compressed if compress else np.savez)(
            path, format=np.int32(_FORMAT), actions=np.int32(ACTIONS), sizes=sizes, **merged)
        return path

    @classmethod
    def load(cls, folder, max_iters=None, device="cpu"):
        h = cls(max_iters)
        with np.load(os.path.join(folder, cls.FILE), allow_pickle=False) as z:
            if int(z["format"]) != _FORMAT or int(z["actions"]) != ACTIONS:
                raise ValueError("unsupported example history file")
            sizes = z["sizes"]
            if not len(sizes) or not sizes.sum():
                return h
            cols = {k: torch.from_numpy(z[k]).to(device) for k in FIELDS}
        off = 0
        for n in sizes.tolist():
            h.append(ExampleSet(*(cols[k][off:off + n] for k in FIELDS)))
            off += n
        return h
