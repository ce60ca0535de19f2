"""tf.summary stand-in: scalars (and image statistics) appended to a JSONL file."""
import json
import os
import time
from contextlib import contextmanager

import numpy as np

_default = None


class SummaryWriter:
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "events.jsonl")
        self._f = open(self.path, "a")

    def scalar(self, name, value, step):
        self._f.write(json.dumps({"t": time.time(), "step": int(step), "tag": name, "value": float(value)}) + "\n")

    def image(self, name, data, step):
        a = np.asarray(data, dtype=np.float32)
        self._f.write(json.dumps({"t": time.time(), "step": int(step), "tag": name, "image_shape": list(a.shape),
                                  "mean": float(a.mean()), "std": float(a.std())}) + "\n")

    def flush(self):
        self._f.flush()

    @contextmanager
    def as_default(self):
        global _default
        prev, _default = _default, self
        try:
            yield self
        finally:
            _default = prev


def create_file_writer(logdir):
    return SummaryWriter(logdir)
