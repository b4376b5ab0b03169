"""rsos_hip -- host-side mirror of reconcile-rs's fingerprint path over librsos_hip.so.

Mirrors the reference's interfaces for this path (names, argument meaning, error
behaviour), so callers and tests read like the reference's own:

  Fingerprint          rsos::Fingerprint         rsos/src/fingerprint.rs:62-228
  Aggregate            rsos::Aggregate           rsos/src/aggregate.rs:38-89
  lift_records         rsos::lift, batched       rsos/src/fingerprint.rs:270-275
  GpuFingerprintStore  rsos::Rsos<K> realisation rsos/src/rsos_trait.rs:39-129
                       (size / aggregate / rank / select / enumerate / insert / delete),
                       which rbsr consumes as RsosView<K> (rbsr/src/rsos_view.rs:55-91)
  FingerprintMap       the same with the host owning K and V and single-record updates staged
                       into one device batch (the Rust binding's HipFingerprintMap)

All hashing runs in the HIP kernels of librsos_hip.so; nothing here computes a
fingerprint on the CPU.  torch is used only for device memory and streams.
"""
from __future__ import annotations

from .fingerprint import Aggregate, Fingerprint
from .schema import RecordSchema
from .device import (lift_records, lift_dual, lift_encoded, lift_fixed, reduce_blocks, range_aggregates,
                     combine_aggregates, block_sums_for)
from .store import GpuFingerprintStore
from .fmap import Entry, FingerprintMap
from ._abi import RsosHipError, lib

__all__ = [
    "Aggregate", "Fingerprint", "RecordSchema", "lift_records", "lift_dual", "lift_encoded", "lift_fixed",
    "reduce_blocks", "range_aggregates", "combine_aggregates", "block_sums_for",
    "GpuFingerprintStore", "FingerprintMap", "Entry", "RsosHipError", "lib",
]
