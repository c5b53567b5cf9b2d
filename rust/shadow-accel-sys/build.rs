// Link against the prebuilt libshd_accel.so (python -m shadow_amd.build).  The crate holds
// declarations only (src/lib.rs, generated from include/shd_accel.h by tools/gen_abi.py).
fn main() {
    let dir = std::env::var("SHD_ACCEL_LIB_DIR").expect("set SHD_ACCEL_LIB_DIR to the directory of libshd_accel.so");
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=shd_accel");
    println!("cargo:rerun-if-env-changed=SHD_ACCEL_LIB_DIR");
}
