//! Links libtpz_gpu.so (built by `make -C topazdb_amd/csrc`, or `__graft_entry__.build()`).
//! TPZ_GPU_LIB_DIR names the directory holding it (default: topazdb_amd/ of this repository).
fn main() {
    let dir = std::env::var("TPZ_GPU_LIB_DIR").unwrap_or_else(|_| {
        let here = std::path::PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap());
        here.join("../../topazdb_amd").display().to_string()
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=tpz_gpu");
    println!("cargo:rerun-if-env-changed=TPZ_GPU_LIB_DIR");
    println!("cargo:rerun-if-changed=../../include/tpz_gpu.h");
}
