//! Links libmdgpu.so (built by `make -C metabodecon-rust_amd ARCH=gfx950`).
//! MDGPU_LIB_DIR overrides the directory; the default is the in-tree build.
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = env::var("MDGPU_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap())
            .join("../../metabodecon-rust_amd/metabodecon")
    });
    println!("cargo:rerun-if-env-changed=MDGPU_LIB_DIR");
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=mdgpu");
    // libmdgpu needs the ROCm HIP runtime at load time
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rustc-link-arg=-Wl,-rpath,/opt/rocm/lib");
}
