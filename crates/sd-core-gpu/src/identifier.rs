//! The batched `identifier_job_step` (core/src/object/file_identifier/
//! mod.rs:100-336) over libsdgpu: one call reads and hashes a whole batch of
//! orphan rows (`sdgpu_identify_files`, replacing the join_all of
//! FileMetadata::new, mod.rs:107-134), one groups them against the library's
//! Objects (`sdgpu_dedup_batch` with an Object index: the find_many of
//! mod.rs:168-185, the link of :189-225, the creates of :233-297).  The write
//! set then becomes one `create_many` + one batched `file_path` update
//! (core/crates/sync/src/manager.rs:62-97) instead of 4-5 queries per 100 rows.
//!
//! Ranks: row i of a step has rank `first_rank + i` -- its position in the
//! job's ascending-id order (file_identifier_job.rs:286-309), i.e. `step *
//! 100 + k` in the reference's terms.  rep[i] == rank: create an Object;
//! rep[i] & SDGPU_REP_EXISTING: connect to the existing Object `rep & 0x7fff_ffff`;
//! otherwise connect to the Object created for the row of rank rep[i].

use std::{io, os::raw::c_char, path::PathBuf, ptr};

use sdgpu_sys as sys;

use crate::{check, cpath, Gpu};

/// One row's outcome (FileMetadata's cas_id + the Object decision).
pub enum Link {
    /// cas_id None (empty file, mod.rs:80-88) or a first sighting: new Object.
    Create,
    /// an Object that existed before the job (caller's handle, e.g. object.id).
    Existing(u32),
    /// the Object created for the row of this rank (this step or an earlier one).
    Row(u32),
    /// metadata / read failed: the row stays an orphan (mod.rs:113,127).
    Failed(io::Error),
}

pub struct IdentifiedRow {
    pub cas_id: Option<String>,
    pub link: Link,
}

/// The library-wide Object index of one job (mod.rs:168-185).
pub struct ObjectIndex(*mut sys::sdgpu_index);
unsafe impl Send for ObjectIndex {}

impl ObjectIndex {
    pub fn new(gpu: &Gpu, capacity: u64) -> io::Result<Self> {
        let mut idx = ptr::null_mut();
        check(unsafe { sys::sdgpu_index_create(*gpu.ctx(), capacity, &mut idx) })?;
        Ok(ObjectIndex(idx))
    }
}

impl Drop for ObjectIndex {
    fn drop(&mut self) {
        unsafe { sys::sdgpu_index_destroy(self.0) };
    }
}

/// One job step over `paths` (rows in id order; `sizes` from fs::metadata,
/// mod.rs:65) whose first row has rank `first_rank`.
pub fn identify_step(gpu: &Gpu, idx: &ObjectIndex, paths: &[PathBuf], sizes: &[u64],
                     first_rank: u32) -> io::Result<Vec<IdentifiedRow>> {
    let n = paths.len();
    let c: Vec<_> = paths.iter().map(|p| cpath(p)).collect();
    let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
    let mut cas8 = vec![[0u8; 8]; n];
    let mut has_key = vec![0u8; n];
    let mut status = vec![0i32; n];
    let mut rep = vec![0u32; n];
    let ctx = gpu.ctx();
    check(unsafe {
        sys::sdgpu_identify_files(*ctx, ptrs.as_ptr(), sizes.as_ptr(), n as u32, cas8.as_mut_ptr(),
                                  has_key.as_mut_ptr(), status.as_mut_ptr())
    })?;
    // rows whose read failed take no part in the grouping (they stay orphans)
    let grouped: Vec<u8> = has_key.iter().zip(&status).map(|(&h, &s)| (h != 0 && s == 0) as u8).collect();
    let keys: Vec<u64> = cas8.iter().map(|b| u64::from_le_bytes(*b)).collect();
    check(unsafe {
        sys::sdgpu_dedup_batch(*ctx, idx.0, keys.as_ptr(), grouped.as_ptr(), first_rank, n as u32,
                               sys::SDGPU_IDENTIFIER_CHUNK_SIZE, rep.as_mut_ptr())
    })?;
    Ok((0..n)
        .map(|i| {
            if status[i] != 0 {
                return IdentifiedRow { cas_id: None, link: Link::Failed(check(status[i]).unwrap_err()) };
            }
            let cas_id = (has_key[i] != 0).then(|| hex::encode(cas8[i]));
            let r = first_rank + i as u32;
            let link = if rep[i] == r {
                Link::Create
            } else if rep[i] & sys::SDGPU_REP_EXISTING != 0 {
                Link::Existing(rep[i] & !sys::SDGPU_REP_EXISTING)
            } else {
                Link::Row(rep[i])
            };
            IdentifiedRow { cas_id, link }
        })
        .collect())
}
