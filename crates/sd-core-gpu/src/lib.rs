//! sd-core's side of the drop-in boundary, over the
//! raw `sdgpu-sys` FFI.  The reference functions keep their signatures:
//!
//! * `generate_cas_id(path, size)` -- core/src/object/cas.rs:23 (body: `cas.rs` here)
//! * `file_checksum(path)`         -- core/src/object/validation/hash.rs:10 (`hash.rs` here)
//! * the grouping / write set of `identifier_job_step`
//!   -- core/src/object/file_identifier/mod.rs:100-336 (`identifier.rs` here)
//!
//! Blocking library calls run inside `spawn_blocking`, as the reference's
//! `tokio::fs` calls do, so the async runtime never blocks.  Errors are the
//! library's `-errno`, mapped with `io::Error::from_raw_os_error` (plus
//! ENODATA -> UnexpectedEof for `read_exact`'s short file, cas.rs:38-57).
//!
//! Not compiled in this repository (the image has no Rust toolchain); the
//! symbols it calls are checked against include/sdgpu.h by tests/test_abi.py.

pub mod burst;
pub mod cas;
pub mod hash;
pub mod identifier;
pub mod job;

use std::{
    ffi::{CStr, CString},
    io,
    os::{raw::c_char, unix::ffi::OsStrExt},
    path::Path,
    sync::{Arc, Mutex, OnceLock},
};

use sdgpu_sys as sys;

/// One libsdgpu context (one GPU), shared by the job system.  The reference
/// runs one job at a time (core/src/job/manager.rs:32); the mutex serialises
/// the watcher's single-file calls against it.
pub struct Gpu(Mutex<*mut sys::sdgpu_ctx>);
unsafe impl Send for Gpu {}
unsafe impl Sync for Gpu {}

static GLOBAL: OnceLock<Arc<Gpu>> = OnceLock::new();
static COALESCER: OnceLock<burst::Coalescer> = OnceLock::new();

/// Opened once at `Node::new` (core/src/lib.rs:77); the drop-ins use it.
pub fn init_global(device: i32) -> io::Result<()> {
    let g = Arc::new(Gpu::open(device)?);
    let _ = GLOBAL.set(g);
    Ok(())
}

pub fn global() -> Arc<Gpu> {
    GLOBAL.get().expect("sd_core_gpu::init_global not called").clone()
}

/// The single-file callers' front door (burst.rs): per-call CPU / GPU policy
/// and coalescing of concurrent calls into one batch.
pub fn coalescer() -> &'static burst::Coalescer {
    COALESCER.get_or_init(|| burst::Coalescer::new(global()))
}

pub(crate) fn check(rc: i32) -> io::Result<()> {
    match rc {
        0 => Ok(()),
        rc if rc == -libc::ENODATA => Err(io::ErrorKind::UnexpectedEof.into()),
        rc => Err(io::Error::from_raw_os_error(-rc)),
    }
}

pub(crate) fn cpath(p: &Path) -> CString {
    CString::new(p.as_os_str().as_bytes()).expect("nul byte in path")
}

impl Gpu {
    pub fn open(device: i32) -> io::Result<Self> {
        let mut ctx = std::ptr::null_mut();
        check(unsafe { sys::sdgpu_open(device, &mut ctx) })?;
        if unsafe { sys::sdgpu_abi_version() } != sys::SDGPU_ABI_VERSION {
            unsafe { sys::sdgpu_close(ctx) };
            return Err(io::Error::new(io::ErrorKind::Other, "libsdgpu ABI version mismatch"));
        }
        Ok(Gpu(Mutex::new(ctx)))
    }

    pub(crate) fn ctx(&self) -> std::sync::MutexGuard<'_, *mut sys::sdgpu_ctx> {
        self.0.lock().unwrap()
    }

    /// `generate_cas_id` of one file: the reference's reads (cas.rs:31-58),
    /// the hash on the GPU, 16 lowercase hex chars.
    pub fn cas_id(&self, path: &Path, size: u64) -> io::Result<String> {
        let mut hex = [0 as c_char; 17];
        let ctx = self.ctx();
        check(unsafe { sys::sdgpu_generate_cas_id(*ctx, cpath(path).as_ptr(), size, hex.as_mut_ptr()) })?;
        Ok(unsafe { CStr::from_ptr(hex.as_ptr()) }.to_string_lossy().into_owned())
    }

    /// `file_checksum` of one file: 64 lowercase hex chars (hash.rs:21-23).
    pub fn checksum(&self, path: &Path) -> io::Result<String> {
        let mut hex = [0 as c_char; 65];
        let ctx = self.ctx();
        check(unsafe { sys::sdgpu_file_checksum(*ctx, cpath(path).as_ptr(), hex.as_mut_ptr()) })?;
        Ok(unsafe { CStr::from_ptr(hex.as_ptr()) }.to_string_lossy().into_owned())
    }
}

impl Drop for Gpu {
    fn drop(&mut self) {
        unsafe { sys::sdgpu_close(*self.0.lock().unwrap()) };
    }
}
