//! Body of core/src/object/cas.rs with the reference signature kept
//! (`pub async fn generate_cas_id(path: impl AsRef<Path>, size: u64) ->
//! Result<String, io::Error>`, cas.rs:23).  The message layout (size LE ||
//! header || 4 samples || footer, cas.rs:10-58) and the reads are done by
//! libsdgpu (`sdgpu_generate_cas_id`); callers: file_identifier/mod.rs:81,
//! location/non_indexed.rs:161, location/manager/watcher/utils.rs:236,411.

use std::{io, path::Path};

pub async fn generate_cas_id(path: impl AsRef<Path>, size: u64) -> Result<String, io::Error> {
    let path = path.as_ref().to_path_buf();
    let gpu = crate::global();
    tokio::task::spawn_blocking(move || gpu.cas_id(&path, size))
        .await
        .map_err(|e| io::Error::new(io::ErrorKind::Other, e))?
}
