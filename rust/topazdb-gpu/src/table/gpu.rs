//! `SsTable::read_blocks_gpu`: the reference's `read_block` (`src/table.rs:154-164`) for a run
//! of blocks at once, decoded on the MI355X through `tpz_decode_blocks_host`.
//!
//! Drop-in module for topazdb: copy to `src/table/gpu.rs`, add `pub mod gpu;` to
//! `src/table.rs` (a child module may read `SsTable`'s private `file`, `block_metas` and
//! `block_meta_offset`), and add to Cargo.toml:
//!
//! ```toml
//! [dependencies]
//! tpz-gpu-sys = { path = "<this repository>/rust/tpz-gpu-sys" }
//! ```
//!
//! The blocks go in as `FileObject::read` returns them (`src/table/file_object.rs:23-27`, one
//! `pread` of the run) and through the library's chunked H2D -> codec step (snappy / lz4) ->
//! decode + CRC pipeline (`tpz_verify_blocks_host`). The reference's `Block` is a view of the
//! block's own bytes (`src/block.rs:46-65`), so the host needs only the device's verdict and,
//! for snappy / lz4 blocks, the decompressed bytes: each `Arc<Block>` is `Block::from_verified`
//! over a slice of the run (`Bytes`, no copy), or the reference's `Err` for a block the
//! reference rejects. `decode_host` (the columns in host memory, `Block::from_columns`) stays
//! for consumers of the decoded keys and values themselves.
use std::ffi::CStr;
use std::os::raw::c_char;
use std::sync::Arc;

use anyhow::{anyhow, bail, Result};
use bytes::Bytes;
use tpz_gpu_sys as ffi;

use super::SsTable;
use crate::block::gpu::HostDecode;
use crate::block::Block;

/// One `tpz_ctx` on one device; shared by any number of threads (calls from different threads
/// use the library's per-call host pipelines).
pub struct GpuDecoder {
    ctx: *mut ffi::TpzCtx,
}

unsafe impl Send for GpuDecoder {}
unsafe impl Sync for GpuDecoder {}

impl GpuDecoder {
    pub fn new(device: i32) -> Result<Self> {
        let abi = unsafe { ffi::tpz_abi_version() };
        if abi != ffi::TPZ_ABI_VERSION {
            bail!("libtpz_gpu ABI {abi}, binding built for {}", ffi::TPZ_ABI_VERSION);
        }
        let mut ctx = std::ptr::null_mut();
        check(unsafe { ffi::tpz_ctx_create(device, &mut ctx) }, "tpz_ctx_create")?;
        Ok(Self { ctx })
    }

    /// tpz_decode_blocks_host over `n` blocks of `region` (`ext` holds n + 1 offsets), growing
    /// the output buffers until every block fits (the call returns TPZ_ERR_NOMEM with the
    /// sizes it needs: h_first[n] pairs, *h_spill_used bytes, h_dext[n] decoded bytes).
    pub fn decode_host(&self, region: &[u8], ext: &[u64]) -> Result<HostDecode> {
        let n = ext.len() - 1;
        let mut bound = 0u64;
        check(unsafe { ffi::tpz_host_decoded_bound(region.as_ptr(), ext.as_ptr(), n as u32, &mut bound) },
              "tpz_host_decoded_bound")?;
        let mut out = HostDecode {
            data: vec![0; unsafe { ffi::tpz_layout_data_capacity(bound, n as u64) } as usize],
            ends: vec![0; 2 * unsafe { ffi::tpz_layout_entry_capacity(bound, n as u64) } as usize],
            first: vec![0; n + 1],
            count: vec![0; n],
            status: vec![0; n],
            crc: vec![0; n],
            spill: Vec::new(),
            spill_off: vec![0; n],
            spill_used: 0,
            dext: vec![0; n + 1],
        };
        loop {
            let cols = ffi::TpzHostColumns {
                h_data: out.data.as_mut_ptr(),
                h_ends: out.ends.as_mut_ptr(),
                ends_cap: out.ends.len() as u64,
                h_first: out.first.as_mut_ptr(),
                h_count: out.count.as_mut_ptr(),
                h_status: out.status.as_mut_ptr(),
                h_crc: out.crc.as_mut_ptr(),
                h_spill: if out.spill.is_empty() { std::ptr::null_mut() } else { out.spill.as_mut_ptr() },
                spill_cap: out.spill.len() as u64,
                h_spill_off: out.spill_off.as_mut_ptr(),
                h_spill_used: &mut out.spill_used,
                h_dext: out.dext.as_mut_ptr(),
                data_cap: out.data.len() as u64,
            };
            let rc = unsafe {
                ffi::tpz_decode_blocks_host(self.ctx, region.as_ptr(), ext.as_ptr(), n as u32, &cols, 0)
            };
            match rc {
                ffi::TPZ_SUCCESS => return Ok(out),
                ffi::TPZ_ERR_NOMEM => {
                    let pairs = out.first[n] as usize;
                    let data = unsafe { ffi::tpz_layout_data_capacity(out.dext[n], n as u64) } as usize;
                    let before = (out.ends.len(), out.spill.len(), out.data.len());
                    out.ends.resize(out.ends.len().max(2 * pairs), 0);
                    out.spill.resize(out.spill.len().max(out.spill_used as usize), 0);
                    out.data.resize(out.data.len().max(data), 0);
                    if before == (out.ends.len(), out.spill.len(), out.data.len()) {
                        bail!("tpz_decode_blocks_host: NOMEM with every buffer at the size it asked for");
                    }
                }
                e => check(e, "tpz_decode_blocks_host")?,
            }
        }
    }
}

/// `tpz_verify_blocks_host`'s outputs for a run of blocks.
pub struct HostVerify {
    pub status: Vec<u8>,
    pub crc: Vec<u32>,
    pub count: Vec<u32>,
    /// the decoded extents and bytes (every block's Uncompress form) when the run holds snappy /
    /// lz4 blocks; `None` when the run itself is the Uncompress form
    pub plain: Option<(Vec<u64>, Bytes)>,
}

impl GpuDecoder {
    /// The device's verdict on `n` blocks of `region` (`ext` holds n + 1 offsets), the decoded
    /// columns left on the device; for a run with snappy / lz4 blocks also their decompressed
    /// bytes (grown until they fit: TPZ_ERR_NOMEM returns the size needed in h_dext[n]).
    pub fn verify_host(&self, region: &[u8], ext: &[u64]) -> Result<HostVerify> {
        let n = ext.len() - 1;
        let codec = (0..n).any(|i| ext[i + 1] > ext[i] && matches!(region[ext[i + 1] as usize - 1], 2 | 3));
        let mut out = HostVerify { status: vec![0; n], crc: vec![0; n], count: vec![0; n], plain: None };
        let mut dext = vec![0u64; n + 1];
        let mut plain: Vec<u8> = Vec::new();
        if codec {
            let mut bound = 0u64;
            check(unsafe { ffi::tpz_host_decoded_bound(region.as_ptr(), ext.as_ptr(), n as u32, &mut bound) },
                  "tpz_host_decoded_bound")?;
            plain.resize(bound as usize, 0);
        }
        loop {
            let rc = unsafe {
                ffi::tpz_verify_blocks_host(self.ctx, region.as_ptr(), ext.as_ptr(), n as u32,
                                            out.status.as_mut_ptr(), out.crc.as_mut_ptr(),
                                            out.count.as_mut_ptr(),
                                            if codec { plain.as_mut_ptr() } else { std::ptr::null_mut() },
                                            plain.len() as u64, dext.as_mut_ptr(), 0)
            };
            match rc {
                ffi::TPZ_SUCCESS => break,
                // NOMEM: h_plain was short and dext[n] holds the bytes needed (grow only then:
                // anything else is an error, never a retry)
                ffi::TPZ_ERR_NOMEM if codec && dext[n] as usize > plain.len() => plain.resize(dext[n] as usize, 0),
                e => check(e, "tpz_verify_blocks_host")?,
            }
        }
        if codec {
            plain.truncate(dext[n] as usize);
            out.plain = Some((dext, Bytes::from(plain)));
        }
        Ok(out)
    }
}

impl Drop for GpuDecoder {
    fn drop(&mut self) {
        unsafe { ffi::tpz_ctx_destroy(self.ctx) };
    }
}

fn check(rc: ffi::TpzErr, what: &str) -> Result<()> {
    if rc == ffi::TPZ_SUCCESS {
        return Ok(());
    }
    let text = unsafe { CStr::from_ptr(ffi::tpz_last_error()) }.to_string_lossy().into_owned();
    Err(anyhow!("{what} failed ({rc}): {text}"))
}

/// The reference's error text for a block status (`checksum.rs:18-21`, `compress.rs:97,102`).
fn block_error(status: u8, expected: u32, actual: u32) -> anyhow::Error {
    let mut buf = [0 as c_char; 128];
    unsafe { ffi::tpz_format_block_error(status as i32, expected, actual, buf.as_mut_ptr(), buf.len()) };
    anyhow!(unsafe { CStr::from_ptr(buf.as_ptr()) }.to_string_lossy().into_owned())
}

impl SsTable {
    /// `read_block` for blocks [first, first + n) in one device call. Each result is what
    /// `read_block(first + i)` returns: `Ok(Arc<Block>)`, the reference's `Err`, or its panic
    /// (`Block::decode` panics on a block too short for its own header, `block.rs:49-59`).
    /// The caller may insert the blocks into the block cache under `(self.id, idx)`, the key
    /// `read_block_cached` uses (`src/table.rs:167-175`).
    pub fn read_blocks_gpu(&self, gpu: &GpuDecoder, first: usize, n: usize) -> Vec<Result<Arc<Block>>> {
        let off = |i: usize| self.block_metas.get(i).map(|m| m.offset).unwrap_or(self.block_meta_offset);
        let lo = off(first);
        // Vec -> Bytes keeps the allocation: every Uncompress block's Block is a slice of it
        let region = match self.file.read(lo, off(first + n) - lo) {
            Ok(r) => Bytes::from(r),
            Err(e) => return (0..n).map(|_| Err(anyhow!("{e}"))).collect(),
        };
        let ext: Vec<u64> = (first..=first + n).map(|i| (off(i) - lo) as u64).collect();
        let v = match gpu.verify_host(&region, &ext) {
            Ok(v) => v,
            Err(e) => return (0..n).map(|_| Err(anyhow!("{e}"))).collect(),
        };
        (0..n)
            .map(|i| match v.status[i] {
                ffi::TPZ_BLOCK_OK | ffi::TPZ_BLOCK_OK_SPILLED | ffi::TPZ_BLOCK_BAD_ENTRY => {
                    let b = match &v.plain {
                        Some((dext, plain)) => plain.slice(dext[i] as usize..dext[i + 1] as usize),
                        None => region.slice(ext[i] as usize..ext[i + 1] as usize),
                    };
                    Ok(Arc::new(Block::from_verified(&b)))
                }
                ffi::TPZ_BLOCK_MALFORMED => panic!("block {} is malformed", first + i),
                st => {
                    // the reference's Err from the device's verdict alone (no CPU decode): a
                    // checksum mismatch names the stored CRC, the big-endian u32 before the tag of
                    // the block's Uncompress form (the run's own bytes, or the device's
                    // decompressed bytes for snappy / lz4, checksum.rs:12-21), and the device's
                    // actual CRC; the other statuses carry no numbers (compress.rs:96-102)
                    let u: &[u8] = match &v.plain {
                        Some((dext, plain)) => &plain[dext[i] as usize..dext[i + 1] as usize],
                        None => &region[ext[i] as usize..ext[i + 1] as usize],
                    };
                    let expected = if st == ffi::TPZ_BLOCK_CHECKSUM_MISMATCH && u.len() >= 5 {
                        u32::from_be_bytes([u[u.len() - 5], u[u.len() - 4], u[u.len() - 3], u[u.len() - 2]])
                    } else {
                        0
                    };
                    Err(block_error(st, expected, v.crc[i]))
                }
            })
            .collect()
    }
}
