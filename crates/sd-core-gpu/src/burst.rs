//! Single-file callers with a per-call policy and burst coalescing
//!.
//!
//! The watcher (core/src/location/manager/watcher/utils.rs:236,411,467) and
//! the non-indexed listing (core/src/location/non_indexed.rs:161) call
//! `generate_cas_id(path, size)` once per file.  One GPU call costs ~23 µs
//! whatever the file (a launch-free resident service, `sdgpu_latency_service`),
//! so a lone small file is hashed on the CPU (the reference's own `blake3`
//! crate, cas.rs:24-61) and a lone large one on the GPU.  When files arrive
//! together -- a folder copied into a watched location, a listing of a new
//! directory -- the requests queued while the worker is busy leave as ONE
//! `sdgpu_identify_files` batch: the reads go to the library's pool and one K1
//! launch hashes them all (bench.py `single_file_latency.burst`).
//!
//! No timer-based linger: the worker drains whatever is queued when it looks,
//! so a lone call waits for nothing and batches grow with the arrival rate.
//!
//! Policy (per request group the worker drains):
//!   * 1 request, message < CPU_BELOW bytes           -> CPU (`blake3` crate)
//!   * 1 request, larger                               -> GPU service
//!   * >= BATCH_FROM requests                           -> one identify_files batch
//!   * size 0 (non_indexed.rs:161 hashes 8 zero bytes)  -> CPU
//! CPU_BELOW and BATCH_FROM come from the measured crossover (include/sdgpu.h,
//! `sdgpu_latency_service`; bench.py burst leg).

use std::{
    io,
    path::PathBuf,
    sync::{mpsc, Arc},
    thread,
};

use tokio::sync::oneshot;

use crate::{check, cpath, sys, Gpu};

/// Messages below this many bytes are hashed on the CPU when they arrive
/// alone (size LE || content: files < ~20 KiB; sdgpu.h's crossover).
pub const CPU_BELOW: u64 = 20 << 10;
/// Requests drained together at or above this count go out as one batch.
pub const BATCH_FROM: usize = 4;
/// Largest batch (the worker drains at most this many at once).
pub const BATCH_MAX: usize = 1024;

struct Req {
    path: PathBuf,
    size: u64,
    reply: oneshot::Sender<io::Result<String>>,
}

/// A worker thread in front of one GPU context.
pub struct Coalescer {
    tx: mpsc::Sender<Req>,
}

/// The cas message length of a file of `size` bytes (cas.rs:10-21).
fn message_len(size: u64) -> u64 {
    if size <= sys::SDGPU_CAS_MINIMUM_FILE_SIZE as u64 {
        8 + size
    } else {
        sys::SDGPU_CAS_SAMPLED_MSG_LEN as u64
    }
}

fn hex16(b: &[u8; 8]) -> String {
    b.iter().map(|x| format!("{x:02x}")).collect()
}

impl Coalescer {
    pub fn new(gpu: Arc<Gpu>) -> Self {
        let (tx, rx) = mpsc::channel::<Req>();
        thread::Builder::new()
            .name("sd-gpu-cas".into())
            .spawn(move || worker(gpu, rx))
            .expect("spawn sd-gpu-cas");
        Coalescer { tx }
    }

    /// `generate_cas_id(path, size)` (cas.rs:23) through the policy above.
    pub async fn cas_id(&self, path: PathBuf, size: u64) -> io::Result<String> {
        let (reply, rx) = oneshot::channel();
        self.tx
            .send(Req { path, size, reply })
            .map_err(|_| io::Error::new(io::ErrorKind::Other, "sd-gpu-cas worker gone"))?;
        rx.await.map_err(|e| io::Error::new(io::ErrorKind::Other, e))?
    }
}

fn worker(gpu: Arc<Gpu>, rx: mpsc::Receiver<Req>) {
    // the service is worth keeping warm only while single large files come in;
    // the library stops it by itself 20 ms after the last call
    while let Ok(first) = rx.recv() {
        let mut group = vec![first];
        while group.len() < BATCH_MAX {
            match rx.try_recv() {
                Ok(r) => group.push(r),
                Err(_) => break,
            }
        }
        if group.len() >= BATCH_FROM {
            batch(&gpu, group);
            continue;
        }
        for r in group {
            let res = if r.size == 0 || message_len(r.size) < CPU_BELOW {
                cpu_cas_id(&r.path, r.size)
            } else {
                gpu.service_cas_id(&r.path, r.size)
            };
            let _ = r.reply.send(res);
        }
    }
}

/// One sdgpu_identify_files call for the whole group (the library's read
/// pool + one K1 launch); size-0 files keep the reference's hash of 8 zero
/// bytes (identify_files treats them as the identifier does: no cas_id).
fn batch(gpu: &Gpu, group: Vec<Req>) {
    let n = group.len();
    let cpaths: Vec<_> = group.iter().map(|r| cpath(&r.path)).collect();
    let ptrs: Vec<_> = cpaths.iter().map(|c| c.as_ptr()).collect();
    let sizes: Vec<u64> = group.iter().map(|r| r.size).collect();
    let mut out8 = vec![[0u8; 8]; n];
    let mut has = vec![0u8; n];
    let mut status = vec![0i32; n];
    let rc = {
        let ctx = gpu.ctx();
        unsafe {
            sys::sdgpu_identify_files(*ctx, ptrs.as_ptr(), sizes.as_ptr(), n as u32,
                                      out8.as_mut_ptr(), has.as_mut_ptr(), status.as_mut_ptr())
        }
    };
    for (i, r) in group.into_iter().enumerate() {
        let res = if rc != 0 {
            check(rc).map(|_| String::new())
        } else if r.size == 0 {
            cpu_cas_id(&r.path, 0)
        } else if status[i] != 0 {
            check(status[i]).map(|_| String::new())
        } else {
            Ok(hex16(&out8[i]))
        };
        let _ = r.reply.send(res);
    }
}

/// The reference's own CPU path (cas.rs:23-62, `blake3` 1.4.1) for small
/// lone files.
fn cpu_cas_id(path: &std::path::Path, size: u64) -> io::Result<String> {
    use std::io::{Read, Seek, SeekFrom};
    let mut hasher = blake3::Hasher::new();
    hasher.update(&size.to_le_bytes());
    if size <= sys::SDGPU_CAS_MINIMUM_FILE_SIZE as u64 {
        hasher.update(&std::fs::read(path)?);
    } else {
        let hf = sys::SDGPU_CAS_HEADER_OR_FOOTER_SIZE as u64;
        let ss = sys::SDGPU_CAS_SAMPLE_SIZE as usize;
        let mut f = std::fs::File::open(path)?;
        let mut head = vec![0u8; hf as usize];
        f.read_exact(&mut head)?;
        hasher.update(&head);
        let jump = (size - 2 * hf) / sys::SDGPU_CAS_SAMPLE_COUNT as u64;
        let mut buf = vec![0u8; ss];
        for k in 0..sys::SDGPU_CAS_SAMPLE_COUNT as u64 {
            f.seek(SeekFrom::Start(hf + k * jump))?;
            f.read_exact(&mut buf)?;
            hasher.update(&buf);
        }
        f.seek(SeekFrom::End(-(hf as i64)))?;
        f.read_exact(&mut head)?;
        hasher.update(&head);
    }
    Ok(hasher.finalize().to_hex()[..16].to_string())
}

impl Gpu {
    /// One file through the resident latency service (enabled on first use).
    pub fn service_cas_id(&self, path: &std::path::Path, size: u64) -> io::Result<String> {
        {
            let ctx = self.ctx();
            check(unsafe { sys::sdgpu_latency_service(*ctx, 1) })?;
        }
        self.cas_id(path, size)
    }
}
