//! Body of core/src/object/validation/hash.rs with the reference signature
//! kept (`pub async fn file_checksum(path: impl AsRef<Path>) -> Result<String,
//! io::Error>`, hash.rs:10): full-file BLAKE3, streamed by libsdgpu in 64 MiB
//! power-of-two slices (`sdgpu_file_checksum`).  `validate_batch` is the
//! batched object-validator step (validator_job.rs:126-169 checksums one file
//! per step): `sdgpu_checksum_files`, where a failed file fails the job
//! (validator_job.rs:147-149).

use std::{io, os::raw::c_char, path::Path, path::PathBuf, sync::Arc};

use sdgpu_sys as sys;

use crate::{check, cpath, Gpu};

pub async fn file_checksum(path: impl AsRef<Path>) -> Result<String, io::Error> {
    let path = path.as_ref().to_path_buf();
    let gpu = crate::global();
    tokio::task::spawn_blocking(move || gpu.checksum(&path))
        .await
        .map_err(|e| io::Error::new(io::ErrorKind::Other, e))?
}

pub async fn validate_batch(gpu: Arc<Gpu>, paths: Vec<PathBuf>) -> io::Result<Vec<String>> {
    tokio::task::spawn_blocking(move || {
        let c: Vec<_> = paths.iter().map(|p| cpath(p)).collect();
        let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
        let mut out = vec![[0u8; 32]; ptrs.len()];
        let mut st = vec![0i32; ptrs.len()];
        let ctx = gpu.ctx();
        check(unsafe {
            sys::sdgpu_checksum_files(*ctx, ptrs.as_ptr(), ptrs.len() as u32, out.as_mut_ptr(),
                                      st.as_mut_ptr())
        })?;
        st.iter().zip(&out).map(|(&s, d)| { check(s)?; Ok(hex::encode(d)) }).collect()
    })
    .await
    .map_err(|e| io::Error::new(io::ErrorKind::Other, e))?
}
