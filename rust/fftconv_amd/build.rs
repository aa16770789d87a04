// Links libfftconv_amd.so (make -C fft-convolution_amd): FFTCONV_AMD_DIR is the
// directory that holds it.
fn main() {
    let dir = std::env::var("FFTCONV_AMD_DIR").unwrap_or_else(|_| "../../fft-convolution_amd".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=fftconv_amd");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=FFTCONV_AMD_DIR");
}
