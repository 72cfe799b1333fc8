//! Body of core/src/object/cas.rs with the reference signature kept
//! (`pub async fn generate_cas_id(path: impl AsRef<Path>, size: u64) ->
//! Result<String, io::Error>`, cas.rs:23).  The message layout (size LE ||
//! header || 4 samples || footer, cas.rs:10-58) and the reads are done by
//! libsdgpu (`sdgpu_generate_cas_id`, or one `sdgpu_identify_files` batch for
//! calls that arrive together, burst.rs); callers: file_identifier/mod.rs:81,
//! location/non_indexed.rs:161, location/manager/watcher/utils.rs:236,411.

use std::{io, path::Path};

pub async fn generate_cas_id(path: impl AsRef<Path>, size: u64) -> Result<String, io::Error> {
    // single-file callers (watcher, non-indexed listing): the coalescer picks
    // CPU or GPU per call and batches concurrent calls (burst.rs); the
    // identifier job does not come here, it batches whole steps
    // (identifier.rs over sdgpu_identify_files)
    crate::coalescer().cas_id(path.as_ref().to_path_buf(), size).await
}
