// Links the prebuilt libsdgpu.so (built by this repository's Makefile).
fn main() {
    let dir = std::env::var("SDGPU_LIB_DIR").unwrap_or_else(|_| "/opt/sdgpu/lib".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=sdgpu");
    println!("cargo:rerun-if-env-changed=SDGPU_LIB_DIR");
}
