// Links librt_hip.so (built by `python -c "import __graft_entry__ as g; g.build()"`).
fn main() {
    let dir = std::env::var("RT_HIP_LIB_DIR").unwrap_or_else(|_| "../bevy_raytrace_amd".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=rt_hip");
    println!("cargo:rerun-if-env-changed=RT_HIP_LIB_DIR");
}
