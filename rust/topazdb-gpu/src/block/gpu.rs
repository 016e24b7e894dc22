//! `Block::from_verified` / `Block::from_columns`: one block of a device decode as the
//! reference's `Block`.
//!
//! Drop-in module for topazdb: copy to `src/block/gpu.rs` and add `pub mod gpu;` to
//! `src/block.rs`. As a child of `block` it may build `Block { data, offsets }`
//! (`src/block.rs:21-24`), whose fields are private to that module; everything that holds an
//! `Arc<Block>` (`BlockIterator`, `SsTableIterator`, `read_block_cached`, `lsm_storage.rs`) then
//! works unchanged.
//!
//! The decode's host outputs (`tpz_decode_blocks_host`, `include/tpz_gpu.h`) hold, per block,
//! its status, entry count, the dense `{kend, vend}` pairs (`h_ends[2 * h_first[i] ..]`: key
//! ends from the stream start, value ends from `tpz_value_start(K)`), and its stream: the slot
//! at `tpz_layout_slot_base(h_dext[i], i)` of `h_data`, or, for `OK_SPILLED` / `BAD_ENTRY`, the
//! spill record at `h_spill + h_spill_off[i]` (stream at `tpz_spill_stream(n)`, and for
//! `BAD_ENTRY` one class byte per entry at `tpz_spill_classes(n, K, V)`).
use bytes::{BufMut, Bytes, BytesMut};
use tpz_gpu_sys as ffi;

use super::Block;

/// The host-side outputs of one `tpz_decode_blocks_host` call (owned buffers).
#[derive(Default)]
pub struct HostDecode {
    pub data: Vec<u8>,
    pub ends: Vec<u32>,
    pub first: Vec<u64>,
    pub count: Vec<u32>,
    pub status: Vec<u8>,
    pub crc: Vec<u32>,
    pub spill: Vec<u8>,
    pub spill_off: Vec<u64>,
    pub spill_used: u64,
    pub dext: Vec<u64>,
}

/// One entry as the reference's iterator would read it from a decoded block.
pub enum EntryView<'a> {
    Ok(&'a [u8], &'a [u8]),
    /// `iterator.rs:81-82` panics on the value; the key is readable (`seek_to_key` reads it)
    BadValue(&'a [u8]),
    /// any read of the entry panics (`iterator.rs:74-80`)
    BadKey,
}

impl HostDecode {
    fn spill_stream(n: u64) -> u64 {
        unsafe { ffi::tpz_layout_spill_stream(n) }
    }

    /// Block i's entries in order (status OK, OK_SPILLED or BAD_ENTRY).
    pub fn entries(&self, i: usize) -> Vec<EntryView<'_>> {
        let n = self.count[i] as usize;
        let pairs = &self.ends[2 * self.first[i] as usize..2 * (self.first[i] as usize + n)];
        let spilled = matches!(self.status[i], ffi::TPZ_BLOCK_OK_SPILLED | ffi::TPZ_BLOCK_BAD_ENTRY);
        let k_tot = if n == 0 { 0 } else { pairs[2 * (n - 1)] as u64 };
        let v_tot = if n == 0 { 0 } else { pairs[2 * (n - 1) + 1] as u64 };
        let vs = ffi::layout::value_start(k_tot) as usize;
        let (stream, classes): (&[u8], Option<&[u8]>) = if spilled {
            let rec = &self.spill[self.spill_off[i] as usize..];
            let s0 = Self::spill_stream(n as u64) as usize;
            let cls = if self.status[i] == ffi::TPZ_BLOCK_BAD_ENTRY {
                let c0 = unsafe { ffi::tpz_layout_spill_classes(n as u64, k_tot, v_tot) } as usize;
                Some(&rec[c0..c0 + n])
            } else {
                None
            };
            (&rec[s0..], cls)
        } else {
            let s = ffi::layout::slot_base(self.dext[i], i as u64) as usize;
            (&self.data[s..], None)
        };
        let (mut k0, mut v0) = (0usize, 0usize);
        (0..n)
            .map(|j| {
                let (k1, v1) = (pairs[2 * j] as usize, pairs[2 * j + 1] as usize);
                let key = &stream[k0..k1];
                let value = &stream[vs + v0..vs + v1];
                k0 = k1;
                v0 = v1;
                match classes.map_or(ffi::TPZ_ENTRY_OK, |c| c[j]) {
                    ffi::TPZ_ENTRY_OK => EntryView::Ok(key, value),
                    ffi::TPZ_ENTRY_BAD_VALUE => EntryView::BadValue(key),
                    _ => EntryView::BadKey,
                }
            })
            .collect()
    }
}

impl Block {
    /// The reference's `Block` from the Uncompress form `b` of a block (payload | crc | tag 1)
    /// whose tag, CRC and header the device has verified (`tpz_verify_blocks_host` status OK,
    /// OK_SPILLED or BAD_ENTRY, so `b.len() >= 7 + 2n`): exactly what `Block::decode(b)` returns
    /// (`src/block.rs:46-65`: `n`, the `n` big-endian offsets, `data` = the payload after them),
    /// with `data` a slice of `b`, no copy. For an Uncompress block `b` is a slice of the bytes
    /// `FileObject::read` returned, for a snappy / lz4 block of the device's decompressed bytes.
    /// A BAD_ENTRY block is the reference's `Ok(Block)` too: its iterator panics by itself on
    /// the out-of-range entries (`iterator.rs:74-82`).
    pub fn from_verified(b: &Bytes) -> Block {
        let n = u16::from_be_bytes([b[0], b[1]]) as usize;
        let offsets = (0..n).map(|j| u16::from_be_bytes([b[2 + 2 * j], b[3 + 2 * j]])).collect();
        Block { data: b.slice(2 + 2 * n..b.len() - 5), offsets }
    }

    /// The reference's `Block` for block i of a device decode (device-column consumers: the
    /// columns are already on the host): `data` holds the entries encoded
    /// as `Entry::encode` writes them (`src/block/builder.rs:72-81`: klen, key, vlen, value;
    /// big-endian u16 lengths) and `offsets` their positions, so `BlockIterator` reads exactly the
    /// keys and values the reference's own `Block::decode` + iterator read from the block bytes.
    ///
    /// A `TPZ_BLOCK_BAD_ENTRY` block is `Ok(Block)` in the reference, whose iterator panics on
    /// the out-of-range entries only (`iterator.rs:74-82`). The rebuilt block keeps that: a
    /// BAD_VALUE entry goes after every readable entry with its key and a value length (0xFFFF)
    /// past the end of `data` (`buf[..vlen]` panics in `seek_to`, while `seek_to_key` can still
    /// compare its key, as in the reference), and a BAD_KEY entry's offset is `data.len()`, where
    /// `get_u16` panics on any read. The device's decode is used as is: no CPU `Block::decode`
    /// of the raw bytes.
    pub fn from_columns(cols: &HostDecode, i: usize) -> Block {
        let ents = cols.entries(i);
        let mut data = BytesMut::new();
        let mut offsets = vec![0u16; ents.len()];
        for (j, e) in ents.iter().enumerate() {
            if let EntryView::Ok(k, v) = e {
                offsets[j] = data.len() as u16;
                data.put_u16(k.len() as u16);
                data.put_slice(k);
                data.put_u16(v.len() as u16);
                data.put_slice(v);
            }
        }
        for (j, e) in ents.iter().enumerate() {
            if let EntryView::BadValue(k) = e {
                offsets[j] = data.len() as u16;
                data.put_u16(k.len() as u16);
                data.put_slice(k);
                data.put_u16(u16::MAX);
            }
        }
        let end = data.len() as u16;
        for (j, e) in ents.iter().enumerate() {
            if let EntryView::BadKey = e {
                offsets[j] = end;
            }
        }
        Block { data: Bytes::from(data), offsets }
    }
}
