"""spacedrive_amd -- MI355X-native content identification for Spacedrive.

Drop-in for sd-core's hot path:
  cas.generate_cas_id            core/src/object/cas.rs:23
  validation.file_checksum       core/src/object/validation/hash.rs:10
  file_identifier.*              core/src/object/file_identifier/mod.rs
  dedup.*                        identifier_job_step's Object grouping
All compute runs in libsdgpu.so (HIP kernels for gfx950); there is no CPU path.
"""
from ._native import Context, SdgpuError, default_context, load  # noqa: F401
from .cas import generate_cas_id  # noqa: F401
from .validation import file_checksum  # noqa: F401

__version__ = "0.1.0"
