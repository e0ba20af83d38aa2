"""pong_amd: the MI355X-native GA evaluation loop behind the reference's
ga.py / main.py surface (n00b001/neuro-genetic-pong-self-play).

  _lib      ctypes binding of libpong_ga.so (include/pong_ga.h)
  device    device-resident Evaluator, Physics and GA operators (torch tensors)
  batched   the batched ``toolbox.map`` that routes ``evaluate`` to one launch
  dist      population sharding over ranks + fitness all-gather
  deap_compat  DEAP's creator/base/tools/algorithms restated (deap is absent)
  build     hipcc build of libpong_ga.so
"""
__version__ = "0.1.0"
