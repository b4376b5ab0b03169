// Link librsos_hip.so.  RSOS_HIP_LIB_DIR points at the directory holding it
// (reconcile-rs_amd/rsos_hip/_lib in the MI355X repository); /opt/rocm/lib provides libamdhip64.
fn main() {
    let dir = std::env::var("RSOS_HIP_LIB_DIR").unwrap_or_else(|_| "/opt/rsos-hip/lib".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=rsos_hip");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rerun-if-env-changed=RSOS_HIP_LIB_DIR");
}
