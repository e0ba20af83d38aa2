"""The reference's policy network (numpy_nn.py:33-137) on the MI355X path.

``NeuralNetwork`` keeps the GA-path API: construction from a flat genome
(``populate_weights``, numpy_nn.py:52-69 layout: one row-major
(out, in + bias) block per layer, bias column last) and ``run(x)`` returning
``[1, 0]`` / ``[0, 1]`` (numpy_nn.py:120-137).  ``run`` is one pg_forward on the
device; batched evaluation never goes through this class (see main.py).

Differences, by design:
  * argmax index >= 2 (3-output networks) returns ``[0, 0]`` (no-op); the
    reference raises "Shouldn't happen" (numpy_nn.py:136-137).
  * only the input and the output entries of ``list_of_transitional_arrays``
    are refreshed by ``run`` (the device does not return hidden activations).
  * backprop training (``train``, numpy_nn.py:84-118) and random init
    (numpy_nn.py:71-82) are not part of the GA path and are not provided.
"""
import logging

import numpy as np
import torch

import config
from pong_amd import runtime

log = logging.getLogger(__name__)


def sigmoid(x):
    """1 / (1 + e**-x), the reference activation (numpy_nn.py:22-23), host-side helper."""
    return 1 / (1 + np.e ** -np.asarray(x, dtype=np.float64))


activation_function = sigmoid


class NeuralNetwork:
    def __init__(self, nodes: list, learning_rate=0.1, bias=None, weights=None):
        self.nodes = list(nodes)
        self.learning_rate = learning_rate
        self.bias = 1 if bias else 0
        self.last_weight = -1 if bias else None
        self.list_of_transitional_arrays = [np.ones(n + self.bias) for n in self.nodes]
        if weights is None:
            raise NotImplementedError("random weight init (numpy_nn.py:71-82) is outside the GA path; "
                                      "pass the genome as weights=")
        self.weights = self.populate_weights(weights)
        used = sum(w.size for w in self.weights)
        self._genes = torch.tensor(np.asarray(weights[:used], dtype=np.float64)[None, :],
                                   device=self._evaluator().device)

    def _evaluator(self):
        return runtime.evaluator(self.nodes, bool(self.bias), genome_dtype="float64",
                                 precision=config.PRECISION, device=config.DEVICE)

    def populate_weights(self, weights):
        """Slice the flat genome into per-layer (out, in + bias) matrices."""
        mats, start = [], 0
        for n_in, n_out in zip(self.nodes[:-1], self.nodes[1:]):
            size = (n_in + self.bias) * n_out
            mats.append(np.array(weights[start:start + size]).reshape(n_out, n_in + self.bias))
            start += size
        if start != len(weights):
            log.warning("Not all weights loaded!\n Loaded: %d weights", start)
        return mats

    def run(self, input_vector):
        n_in = self.nodes[0]
        if len(input_vector) != n_in:
            raise Exception("input vector wrong shape")
        ev = self._evaluator()
        x = torch.tensor(np.asarray(input_vector, dtype=np.float64)[None, :], device=ev.device)
        idx, act = ev.forward(self._genes, x)
        self.list_of_transitional_arrays[0][:n_in] = input_vector
        self.list_of_transitional_arrays[-1][:self.nodes[-1]] = act[0].cpu().numpy()
        i = int(idx[0])
        return [1, 0] if i == 0 else ([0, 1] if i == 1 else [0, 0])
