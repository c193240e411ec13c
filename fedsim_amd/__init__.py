"""fedsim_amd — MI355X-native server aggregation path for FedSim.

The accelerated path: client vectors are packed into HBM and reduced by a
hand-written gfx950 HIP kernel (libfedagg.so, C-ABI in include/fedagg.h),
bit-identical to the reference CPU aggregation.  Entry points mirror the
reference's names:

  fedsim_amd.utils.SerialAggregator                 (fedsim/utils/aggregators.py)
  fedsim_amd.distributed.centralized.training.FedAvg / AdaBest / FedNova
  fedsim_amd.distributed.centralized.CentralFLAlgorithm
"""
__version__ = "0.1.0"
