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

use std::{io, marker::PhantomData, os::raw::c_char, path::PathBuf, ptr};

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

/// The library-wide Object index of one job (mod.rs:168-185).  It borrows
/// its `Gpu`: sdgpu_close frees what the index points into, so the index
/// must be dropped first (include/sdgpu.h, sdgpu_close).
pub struct ObjectIndex<'g>(*mut sys::sdgpu_index, PhantomData<&'g Gpu>);
unsafe impl Send for ObjectIndex<'_> {}

impl<'g> ObjectIndex<'g> {
    pub fn new(gpu: &'g Gpu, capacity: u64) -> io::Result<Self> {
        let mut idx = ptr::null_mut();
        check(unsafe { sys::sdgpu_index_create(*gpu.ctx(), capacity, &mut idx) })?;
        Ok(ObjectIndex(idx, PhantomData))
    }
}

impl Drop for ObjectIndex<'_> {
    fn drop(&mut self) {
        unsafe { sys::sdgpu_index_destroy(self.0) };
    }
}

impl ObjectIndex<'_> {
    /// Objects that exist before the job (mod.rs:168-185): key -> object id.
    pub fn add_objects(&self, gpu: &Gpu, keys: &[u64], ids: &[u32]) -> io::Result<()> {
        if keys.is_empty() {
            return Ok(());
        }
        let ctx = gpu.ctx();
        let n = keys.len();
        let mut dk = ptr::null_mut();
        let mut dh = ptr::null_mut();
        check(unsafe { sys::sdgpu_alloc_device(*ctx, 8 * n, &mut dk) })?;
        check(unsafe { sys::sdgpu_alloc_device(*ctx, 4 * n, &mut dh) })?;
        let stream = unsafe { sys::sdgpu_stream(*ctx) };
        let rc = unsafe {
            check(sys::sdgpu_memcpy_async(*ctx, dk, keys.as_ptr().cast(), 8 * n, stream))
                .and_then(|_| check(sys::sdgpu_memcpy_async(*ctx, dh, ids.as_ptr().cast(), 4 * n, stream)))
                .and_then(|_| check(sys::sdgpu_index_add_objects_device(self.0, dk.cast(), dh.cast(),
                                                                       n as u64, 1, 0, stream)))
                .and_then(|_| check(sys::sdgpu_sync(*ctx)))
        };
        unsafe {
            sys::sdgpu_free_device(*ctx, dk);
            sys::sdgpu_free_device(*ctx, dh);
        }
        rc
    }
}

/// What one batched read + hash of the candidates gives (FileMetadata::new of
/// every row, mod.rs:107-134): cas bytes, has_key, -errno per row.
pub struct Identified {
    pub cas8: Vec<[u8; 8]>,
    pub has_key: Vec<u8>,
    pub status: Vec<i32>,
}

/// `sizes` None: the library stats every path itself (ABI 6), as the
/// reference's FileMetadata::new does (mod.rs:65,80-81).
pub fn identify(gpu: &Gpu, paths: &[PathBuf], sizes: Option<&[u64]>) -> io::Result<Identified> {
    let n = paths.len();
    if sizes.map_or(false, |s| s.len() != n) {
        return Err(io::Error::new(io::ErrorKind::InvalidInput, "one size per path"));
    }
    let c: Vec<_> = paths.iter().map(|p| cpath(p)).collect();
    let ptrs: Vec<*const c_char> = c.iter().map(|s| s.as_ptr()).collect();
    let mut out = Identified { cas8: vec![[0u8; 8]; n], has_key: vec![0u8; n], status: vec![0i32; n] };
    let ctx = gpu.ctx();
    check(unsafe {
        sys::sdgpu_identify_files(*ctx, ptrs.as_ptr(), sizes.map_or(std::ptr::null(), |s| s.as_ptr()),
                                  n as u32, out.cas8.as_mut_ptr(),
                                  out.has_key.as_mut_ptr(), out.status.as_mut_ptr())
    })?;
    Ok(out)
}

/// The grouping of one batch of identified rows against the index (rows in
/// id order, ranks first_rank + i); rows whose read failed take no part.
pub fn group(gpu: &Gpu, idx: &ObjectIndex<'_>, rows: &Identified, first_rank: u32) -> io::Result<Vec<IdentifiedRow>> {
    let n = rows.cas8.len();
    let mut rep = vec![0u32; n];
    let grouped: Vec<u8> =
        rows.has_key.iter().zip(&rows.status).map(|(&h, &s)| (h != 0 && s == 0) as u8).collect();
    let keys: Vec<u64> = rows.cas8.iter().map(|b| u64::from_le_bytes(*b)).collect();
    {
        let ctx = gpu.ctx();
        check(unsafe {
            sys::sdgpu_dedup_batch(*ctx, idx.0, keys.as_ptr(), grouped.as_ptr(), first_rank, n as u32,
                                   sys::SDGPU_IDENTIFIER_CHUNK_SIZE, rep.as_mut_ptr())
        })?;
    }
    Ok((0..n)
        .map(|i| {
            if rows.status[i] != 0 {
                return IdentifiedRow { cas_id: None, link: Link::Failed(check(rows.status[i]).unwrap_err()) };
            }
            let cas_id = (rows.has_key[i] != 0).then(|| hex::encode(rows.cas8[i]));
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

/// One job step over `paths` (rows in id order; `sizes` from fs::metadata,
/// mod.rs:65) whose first row has rank `first_rank`.
pub fn identify_step(gpu: &Gpu, idx: &ObjectIndex<'_>, paths: &[PathBuf], sizes: Option<&[u64]>,
                     first_rank: u32) -> io::Result<Vec<IdentifiedRow>> {
    let rows = identify(gpu, paths, sizes)?;
    group(gpu, idx, &rows, first_rank)
}
