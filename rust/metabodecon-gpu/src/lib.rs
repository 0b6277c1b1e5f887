//! MI355X (gfx950) backend for metabodecon's `Deconvoluter` hot path.
//!
//! A thin `extern "C"` shim over `libmdgpu` (the C ABI of `include/mdgpu.h`)
//! plus safe wrappers that take and return the reference crate's own types
//! (SombkeMaximilian/metabodecon-rust, `metabodecon/src`), so callers switch by
//! calling `gpu_*` instead of the CPU methods and get identical results:
//!
//! | reference (CPU)                                   | here                                   |
//! |---------------------------------------------------|----------------------------------------|
//! | `Deconvoluter::deconvolute_spectrum` (deconvoluter.rs:530-552), `par_deconvolute_spectrum` (:591-613) | [`GpuDeconvoluter::gpu_deconvolute_spectrum`] |
//! | `Deconvoluter::deconvolute_spectra` (:651-661), `par_deconvolute_spectra` (:700-710) | [`GpuDeconvoluter::gpu_deconvolute_spectra`] |
//! | `Deconvoluter::optimize_settings` (:762-825)     | [`GpuDeconvoluter::gpu_optimize_settings`] |
//! | `Lorentzian::superposition_vec` / `par_superposition_vec` (lorentzian.rs:631-663) | [`gpu_superposition_vec`] |
//! | many concurrent `par_deconvolute_spectrum` callers (Deconvoluter is `Send + Sync`, deconvoluter.rs:913-917) | [`GpuSpectrumQueue`] (device arrays, batched internally) |
//!
//! The reference's stage traits are `pub(crate)`, so the seam is these public
//! methods; everything here uses only the reference's public API
//! (`Deconvoluter::{smoothing,selection,fitting}_settings` deconvoluter.rs:229-277,
//! `ignore_regions` :296, `Spectrum::{chemical_shifts, intensities,
//! signal_boundaries}` spectrum.rs:225-275, `Deconvolution::new`
//! deconvolution.rs:75-81, `Lorentzian::new` lorentzian.rs:207), so it builds
//! against the reference crate unchanged. `Lorentzian` is `repr(Rust)`
//! (lorentzian.rs:138-145): the engine returns `repr(C)` triples and the shim
//! rebuilds them with `Lorentzian::new(sfhw, hw2, maxp)`.

use std::ffi::CStr;
use std::os::raw::{c_int, c_void};
use std::ptr::{self, NonNull};
use std::sync::atomic::{AtomicI32, Ordering};

use metabodecon::deconvolution::error::{Error as DeconvolutionError, Kind};
use metabodecon::deconvolution::{
    Deconvoluter, Deconvolution, FittingSettings, Lorentzian, ScoringMethod, SelectionSettings,
    SmoothingSettings,
};
use metabodecon::spectrum::Spectrum;
use metabodecon::{Error, Result};

/// Raw bindings: one declaration per entry point of `include/mdgpu.h`, same
/// order and types (`tests/test_rust_shim_abi.py` compiles these signatures
/// against the header and calls the host-only ones).
pub mod ffi {
    use std::os::raw::{c_char, c_int, c_void};

    /// `mdg_settings` (mdgpu.h): Deconvoluter settings as plain fields.
    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default, PartialEq)]
    pub struct MdgSettings {
        pub smoother: i32,
        pub smooth_iterations: u32,
        pub smooth_window: u32,
        pub selector: i32,
        pub scoring: i32,
        pub fit_iterations: u32,
        pub fitter: i32,
        pub options: i32,
        pub threshold: f64,
    }

    /// `mdg_lorentzian` (mdgpu.h): transformed parameters, repr(C).
    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default, PartialEq)]
    pub struct MdgLorentzian {
        pub sfhw: f64,
        pub hw2: f64,
        pub maxp: f64,
    }

    /// Opaque `mdg_ctx`.
    #[repr(C)]
    pub struct MdgCtx {
        _private: [u8; 0],
    }

    /// Opaque `mdg_queue` (the spectrum queue).
    #[repr(C)]
    pub struct MdgQueue {
        _private: [u8; 0],
    }

    pub const MDG_OK: c_int = 0;
    pub const MDG_NO_PEAKS_DETECTED: c_int = 1;
    pub const MDG_EMPTY_SIGNAL_REGION: c_int = 2;
    pub const MDG_EMPTY_SIGNAL_FREE_REGION: c_int = 3;
    pub const MDG_INVALID_SMOOTHING: c_int = 10;
    pub const MDG_INVALID_SELECTION: c_int = 11;
    pub const MDG_INVALID_FITTING: c_int = 12;
    pub const MDG_INVALID_IGNORE_REGION: c_int = 13;
    pub const MDG_INVALID_ARGUMENT: c_int = 20;
    pub const MDG_CAPACITY: c_int = 21;
    pub const MDG_REFERENCE_PANIC: c_int = 30;

    pub const MDG_SMOOTH_IDENTITY: i32 = 0;
    pub const MDG_SMOOTH_MOVING_AVERAGE: i32 = 1;
    pub const MDG_SELECT_DETECTOR_ONLY: i32 = 0;
    pub const MDG_SELECT_NOISE_SCORE: i32 = 1;
    pub const MDG_SCORE_MINIMUM_SUM: i32 = 0;
    pub const MDG_FIT_ANALYTICAL: i32 = 0;
    pub const MDG_OPTION_EXACT_MSE: i32 = 1;

    #[link(name = "mdgpu")]
    extern "C" {
        pub fn mdg_abi_version() -> c_int;
        pub fn mdg_strerror(status: c_int) -> *const c_char;
        pub fn mdg_settings_default(s: *mut MdgSettings);
        pub fn mdg_settings_validate(s: *const MdgSettings) -> c_int;
        pub fn mdg_ignore_region_add(
            regions: *mut f64,
            n: usize,
            cap: usize,
            a: f64,
            b: f64,
            n_out: *mut usize,
        ) -> c_int;
        pub fn mdg_jcampdx_decode(
            data: *const c_char,
            len: usize,
            factor: f64,
            out: *mut f64,
            cap: usize,
            n_out: *mut usize,
        ) -> c_int;
        pub fn mdg_device_count(count: *mut c_int) -> c_int;
        pub fn mdg_host_alloc(device: c_int, bytes: usize, out: *mut *mut c_void) -> c_int;
        pub fn mdg_host_free(p: *mut c_void) -> c_int;
        pub fn mdg_ctx_create(device: c_int, out: *mut *mut MdgCtx) -> c_int;
        pub fn mdg_ctx_destroy(ctx: *mut MdgCtx) -> c_int;
        pub fn mdg_ctx_set_stream(ctx: *mut MdgCtx, hip_stream: *mut c_void) -> c_int;
        pub fn mdg_ctx_synchronize(ctx: *mut MdgCtx) -> c_int;
        pub fn mdg_ctx_set_latency_mode(ctx: *mut MdgCtx, on: c_int) -> c_int;
        pub fn mdg_ctx_reload_switches(ctx: *mut MdgCtx) -> c_int;
        pub fn mdg_ctx_set_tracing(ctx: *mut MdgCtx, on: c_int) -> c_int;
        pub fn mdg_deconvolute(
            ctx: *mut MdgCtx,
            x: *const f64,
            y: *const f64,
            n: usize,
            sb0: f64,
            sb1: f64,
            s: *const MdgSettings,
            ignore: *const f64,
            n_ignore: usize,
            out: *mut MdgLorentzian,
            cap: usize,
            out_count: *mut usize,
            out_mse: *mut f64,
        ) -> c_int;
        pub fn mdg_deconvolute_batch(
            ctx: *mut MdgCtx,
            b: usize,
            n: usize,
            x: *const f64,
            x_stride: usize,
            y: *const f64,
            y_stride: usize,
            sb: *const f64,
            s: *const MdgSettings,
            ignore: *const f64,
            n_ignore: usize,
            out: *mut MdgLorentzian,
            cap: usize,
            counts: *mut usize,
            mse: *mut f64,
            status: *mut c_int,
        ) -> c_int;
        pub fn mdg_deconvolute_rows(
            ctx: *mut MdgCtx,
            b: usize,
            n: usize,
            x_rows: *const *const f64,
            y_rows: *const *const f64,
            sb: *const f64,
            s: *const MdgSettings,
            ignore: *const f64,
            n_ignore: usize,
            out: *mut MdgLorentzian,
            cap: usize,
            counts: *mut usize,
            mse: *mut f64,
            status: *mut c_int,
        ) -> c_int;
        pub fn mdg_deconvolute_rows_i32(
            ctx: *mut MdgCtx,
            b: usize,
            n: usize,
            axes: *const f64,
            y_rows: *const *const i32,
            y_scale: *const f64,
            sb: *const f64,
            s: *const MdgSettings,
            ignore: *const f64,
            n_ignore: usize,
            out: *mut MdgLorentzian,
            cap: usize,
            counts: *mut usize,
            mse: *mut f64,
            status: *mut c_int,
        ) -> c_int;
        pub fn mdg_deconvolute_batch_device(
            ctx: *mut MdgCtx,
            b: usize,
            n: usize,
            d_x: *const f64,
            x_stride: usize,
            d_y: *const f64,
            y_stride: usize,
            d_sb: *const f64,
            s: *const MdgSettings,
            ignore: *const f64,
            n_ignore: usize,
            d_out: *mut MdgLorentzian,
            cap: usize,
            d_counts: *mut i32,
            d_mse: *mut f64,
            d_status: *mut i32,
        ) -> c_int;
        pub fn mdg_optimize_settings(
            ctx: *mut MdgCtx,
            x: *const f64,
            y: *const f64,
            n: usize,
            sb0: f64,
            sb1: f64,
            ignore: *const f64,
            n_ignore: usize,
            best: *mut MdgSettings,
            best_mse: *mut f64,
        ) -> c_int;
        pub fn mdg_superposition_vec(
            ctx: *mut MdgCtx,
            x: *const f64,
            n: usize,
            l: *const MdgLorentzian,
            p: usize,
            out: *mut f64,
        ) -> c_int;
        pub fn mdg_superposition_vec_device(
            ctx: *mut MdgCtx,
            d_x: *const f64,
            n: usize,
            d_l: *const MdgLorentzian,
            p: usize,
            d_out: *mut f64,
        ) -> c_int;
        pub fn mdg_queue_create(
            device: c_int,
            n: usize,
            max_batch: usize,
            lanes: c_int,
            s: *const MdgSettings,
            ignore: *const f64,
            n_ignore: usize,
            out: *mut *mut MdgQueue,
        ) -> c_int;
        pub fn mdg_queue_submit(
            q: *mut MdgQueue,
            d_x: *const f64,
            d_y: *const f64,
            sb0: f64,
            sb1: f64,
            d_out: *mut MdgLorentzian,
            cap: usize,
            d_count: *mut i32,
            d_mse: *mut f64,
            d_status: *mut i32,
        ) -> c_int;
        pub fn mdg_queue_flush(q: *mut MdgQueue) -> c_int;
        pub fn mdg_queue_set_flush_us(q: *mut MdgQueue, us: i64) -> c_int;
        pub fn mdg_queue_synchronize(q: *mut MdgQueue) -> c_int;
        pub fn mdg_queue_lane(q: *mut MdgQueue, lane: c_int, ctx: *mut *mut MdgCtx) -> c_int;
        pub fn mdg_queue_stats(
            q: *mut MdgQueue,
            batches: *mut u64,
            spectra: *mut u64,
            open: *mut usize,
        ) -> c_int;
        pub fn mdg_queue_destroy(q: *mut MdgQueue) -> c_int;
    }
}

/// One device context of the engine: a HIP stream and a reusable HBM workspace.
/// The C context is internally locked (mdgpu.h), so it may be shared by threads
/// like the reference's `Send + Sync` Deconvoluter (deconvoluter.rs:913-917).
pub struct GpuContext {
    ctx: NonNull<ffi::MdgCtx>,
    /// `mdg_settings.options` for the calls made through this context
    /// (`MDG_OPTION_EXACT_MSE`, set by `set_exact_mse`).
    options: AtomicI32,
}

unsafe impl Send for GpuContext {}
unsafe impl Sync for GpuContext {}

impl GpuContext {
    /// Context on HIP device `device`; errors when no MI355X is visible.
    pub fn new(device: i32) -> Result<Self> {
        let mut raw: *mut ffi::MdgCtx = ptr::null_mut();
        let st = unsafe { ffi::mdg_ctx_create(device as c_int, &mut raw) };
        match NonNull::new(raw) {
            Some(ctx) if st == ffi::MDG_OK => Ok(Self { ctx, options: AtomicI32::new(0) }),
            _ => Err(engine_error(st)),
        }
    }

    /// Number of visible HIP devices.
    pub fn device_count() -> usize {
        let mut n: c_int = 0;
        unsafe { ffi::mdg_device_count(&mut n) };
        n.max(0) as usize
    }

    /// Enqueue later work on this `hipStream_t` (null: the context's own stream).
    ///
    /// # Safety
    /// `stream` must be a valid HIP stream of this context's device.
    pub unsafe fn set_stream(&self, stream: *mut c_void) -> Result<()> {
        check(ffi::mdg_ctx_set_stream(self.raw(), stream))
    }

    pub fn synchronize(&self) -> Result<()> {
        check(unsafe { ffi::mdg_ctx_synchronize(self.raw()) })
    }

    /// Engine option (not a reference setting): compute each `Deconvolution`'s MSE in
    /// the reference's summation order (`compute_mse`, deconvoluter.rs:828-862), bit
    /// for bit; off (the default) it is within 1e-12 relative and cheaper. The
    /// Lorentzians are bit-identical either way (mdgpu.h `MDG_OPTION_EXACT_MSE`).
    pub fn set_exact_mse(&self, on: bool) {
        let v = if on { ffi::MDG_OPTION_EXACT_MSE } else { 0 };
        self.options.store(v, Ordering::Relaxed);
    }

    pub fn exact_mse(&self) -> bool {
        self.options.load(Ordering::Relaxed) & ffi::MDG_OPTION_EXACT_MSE != 0
    }

    /// Latency mode (on by default): a one-spectrum call expects the GPU to itself and
    /// takes the fit tiling fastest alone; turn it off on contexts that run
    /// `par_deconvolute_spectrum` callers concurrently. Results are bit-identical.
    pub fn set_latency_mode(&self, on: bool) -> Result<()> {
        check(unsafe { ffi::mdg_ctx_set_latency_mode(self.raw(), on as c_int) })
    }

    fn options(&self) -> i32 {
        self.options.load(Ordering::Relaxed)
    }

    pub fn raw(&self) -> *mut ffi::MdgCtx {
        self.ctx.as_ptr()
    }
}

impl Drop for GpuContext {
    fn drop(&mut self) {
        unsafe { ffi::mdg_ctx_destroy(self.ctx.as_ptr()) };
    }
}

/// The spectrum queue (`mdg_queue_*`): the serving form of many concurrent
/// `Deconvoluter::par_deconvolute_spectrum` calls (the reference's Deconvoluter
/// is `Send + Sync`, deconvoluter.rs:913-917). Each submission is one spectrum in
/// device memory; the engine runs them in batches of `max_batch` on `lanes`
/// engine contexts. Settings and ignore regions are the Deconvoluter's at
/// creation.
pub struct GpuSpectrumQueue {
    q: NonNull<ffi::MdgQueue>,
}

unsafe impl Send for GpuSpectrumQueue {}
unsafe impl Sync for GpuSpectrumQueue {}

impl GpuSpectrumQueue {
    /// Queue for spectra of `n` points on HIP device `device`.
    pub fn new(
        deconvoluter: &Deconvoluter,
        device: i32,
        n: usize,
        max_batch: usize,
        lanes: i32,
    ) -> Result<Self> {
        Self::with_exact_mse(deconvoluter, device, n, max_batch, lanes, false)
    }

    /// `new`, with the exact-order MSE option (`GpuContext::set_exact_mse`).
    pub fn with_exact_mse(
        deconvoluter: &Deconvoluter,
        device: i32,
        n: usize,
        max_batch: usize,
        lanes: i32,
        exact_mse: bool,
    ) -> Result<Self> {
        let options = if exact_mse { ffi::MDG_OPTION_EXACT_MSE } else { 0 };
        let s = Settings::of(deconvoluter).to_ffi(options)?;
        let ig = ignore_pairs(deconvoluter);
        let mut raw: *mut ffi::MdgQueue = ptr::null_mut();
        let st = unsafe {
            ffi::mdg_queue_create(
                device as c_int,
                n,
                max_batch,
                lanes as c_int,
                &s,
                opt_ptr(&ig),
                ig.len() / 2,
                &mut raw,
            )
        };
        match NonNull::new(raw) {
            Some(q) if st == ffi::MDG_OK => Ok(Self { q }),
            _ => Err(engine_error(st)),
        }
    }

    /// Submit one spectrum (asynchronous).
    ///
    /// # Safety
    /// Every pointer is device memory of the queue's device: `d_x`, `d_y` hold `n`
    /// values and stay unchanged, and `d_out` (`cap` entries), `d_count`, `d_mse`,
    /// `d_status` stay valid, until [`GpuSpectrumQueue::synchronize`] returns.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn submit(
        &self,
        d_x: *const f64,
        d_y: *const f64,
        signal_boundaries: (f64, f64),
        d_out: *mut ffi::MdgLorentzian,
        cap: usize,
        d_count: *mut i32,
        d_mse: *mut f64,
        d_status: *mut i32,
    ) -> Result<()> {
        check(ffi::mdg_queue_submit(
            self.q.as_ptr(),
            d_x,
            d_y,
            signal_boundaries.0,
            signal_boundaries.1,
            d_out,
            cap,
            d_count,
            d_mse,
            d_status,
        ))
    }

    /// Launch the open (partial) batch.
    pub fn flush(&self) -> Result<()> {
        check(unsafe { ffi::mdg_queue_flush(self.q.as_ptr()) })
    }

    /// Launch the open batch once its first submission has waited `us`
    /// microseconds (0: only full batches and explicit flushes launch).
    pub fn set_flush_us(&self, us: i64) -> Result<()> {
        check(unsafe { ffi::mdg_queue_set_flush_us(self.q.as_ptr(), us) })
    }

    /// Flush and wait until every submission's outputs are written.
    pub fn synchronize(&self) -> Result<()> {
        check(unsafe { ffi::mdg_queue_synchronize(self.q.as_ptr()) })
    }
}

impl Drop for GpuSpectrumQueue {
    fn drop(&mut self) {
        unsafe { ffi::mdg_queue_destroy(self.q.as_ptr()) };
    }
}

fn strerror(status: c_int) -> String {
    let p = unsafe { ffi::mdg_strerror(status) };
    if p.is_null() {
        return format!("mdgpu status {status}");
    }
    unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
}

/// Engine failures (HIP errors, invalid arguments) have no `Kind` in the
/// reference; they surface as the reference's `Error::IoError`.
fn engine_error(status: c_int) -> Error {
    Error::IoError(std::io::Error::new(
        std::io::ErrorKind::Other,
        format!("mdgpu: {}", strerror(status)),
    ))
}

fn check(status: c_int) -> Result<()> {
    if status == ffi::MDG_OK {
        Ok(())
    } else {
        Err(engine_error(status))
    }
}

/// The three settings enums of a Deconvoluter, kept for error reporting.
#[derive(Clone, Copy)]
struct Settings {
    smoothing: SmoothingSettings,
    selection: SelectionSettings,
    fitting: FittingSettings,
}

impl Settings {
    fn of(d: &Deconvoluter) -> Self {
        Self {
            smoothing: d.smoothing_settings(),
            selection: d.selection_settings(),
            fitting: d.fitting_settings(),
        }
    }

    /// The deconvolution-time errors of the reference (deconvolution/error.rs:39-95).
    fn error(&self, status: c_int) -> Error {
        let kind = match status {
            ffi::MDG_NO_PEAKS_DETECTED => Kind::NoPeaksDetected,
            ffi::MDG_EMPTY_SIGNAL_REGION => Kind::EmptySignalRegion,
            ffi::MDG_EMPTY_SIGNAL_FREE_REGION => Kind::EmptySignalFreeRegion,
            ffi::MDG_INVALID_SMOOTHING => Kind::InvalidSmoothingSettings {
                settings: self.smoothing,
            },
            ffi::MDG_INVALID_SELECTION => Kind::InvalidSelectionSettings {
                settings: self.selection,
            },
            ffi::MDG_INVALID_FITTING => Kind::InvalidFittingSettings {
                settings: self.fitting,
            },
            // the reference panics on these inputs (slice bounds in the smoother or
            // compute_mse); so does the shim, instead of inventing an error kind
            ffi::MDG_REFERENCE_PANIC => panic!("{}", strerror(status)),
            _ => return engine_error(status),
        };
        Error::Deconvolution(DeconvolutionError::new(kind))
    }

    /// Enum settings -> `mdg_settings` (smoother.rs:27-65, selector.rs:21-66,
    /// fitter.rs:26-63). Variants the engine does not know are rejected as the
    /// matching invalid-settings error.
    fn to_ffi(&self, options: i32) -> Result<ffi::MdgSettings> {
        let mut s = ffi::MdgSettings::default();
        unsafe { ffi::mdg_settings_default(&mut s) };
        s.options = options;
        let too_big = |v: usize| u32::try_from(v).is_err();
        match self.smoothing {
            SmoothingSettings::Identity => s.smoother = ffi::MDG_SMOOTH_IDENTITY,
            SmoothingSettings::MovingAverage { iterations, window_size }
                if !too_big(iterations) && !too_big(window_size) =>
            {
                s.smoother = ffi::MDG_SMOOTH_MOVING_AVERAGE;
                s.smooth_iterations = iterations as u32;
                s.smooth_window = window_size as u32;
            }
            _ => return Err(self.error(ffi::MDG_INVALID_SMOOTHING)),
        }
        match self.selection {
            SelectionSettings::DetectorOnly => s.selector = ffi::MDG_SELECT_DETECTOR_ONLY,
            SelectionSettings::NoiseScoreFilter {
                scoring_method: ScoringMethod::MinimumSum,
                threshold,
            } => {
                s.selector = ffi::MDG_SELECT_NOISE_SCORE;
                s.scoring = ffi::MDG_SCORE_MINIMUM_SUM;
                s.threshold = threshold;
            }
            _ => return Err(self.error(ffi::MDG_INVALID_SELECTION)),
        }
        match self.fitting {
            FittingSettings::Analytical { iterations } if !too_big(iterations) => {
                s.fitter = ffi::MDG_FIT_ANALYTICAL;
                s.fit_iterations = iterations as u32;
            }
            _ => return Err(self.error(ffi::MDG_INVALID_FITTING)),
        }
        Ok(s)
    }

    fn deconvolution(&self, params: &[ffi::MdgLorentzian], mse: f64) -> Deconvolution {
        let lorentzians = params
            .iter()
            .map(|p| Lorentzian::new(p.sfhw, p.hw2, p.maxp))
            .collect();
        Deconvolution::new(lorentzians, self.smoothing, self.selection, self.fitting, mse)
    }
}

/// Merged ignore regions as the flat (lo, hi) ppm pairs mdg_* take
/// (`ignore_regions() -> Option<&[(f64, f64)]>`, deconvoluter.rs:296).
fn ignore_pairs(d: &Deconvoluter) -> Vec<f64> {
    d.ignore_regions()
        .map(|r| r.iter().flat_map(|&(a, b)| [a, b]).collect())
        .unwrap_or_default()
}

fn opt_ptr(v: &[f64]) -> *const f64 {
    if v.is_empty() {
        ptr::null()
    } else {
        v.as_ptr()
    }
}

/// The reference's Deconvoluter methods, run on the GPU.
pub trait GpuDeconvoluter {
    /// `deconvolute_spectrum` / `par_deconvolute_spectrum` (deconvoluter.rs:530-613).
    fn gpu_deconvolute_spectrum(&self, ctx: &GpuContext, spectrum: &Spectrum) -> Result<Deconvolution>;

    /// `deconvolute_spectra` / `par_deconvolute_spectra` (deconvoluter.rs:651-710):
    /// one batched pipeline per distinct spectrum length; the first error in input
    /// order is returned, like the reference's `Result` collect.
    fn gpu_deconvolute_spectra<S: AsRef<Spectrum>>(
        &self,
        ctx: &GpuContext,
        spectra: &[S],
    ) -> Result<Vec<Deconvolution>>;

    /// `optimize_settings` (deconvoluter.rs:762-825): the 810-setting grid search;
    /// sets the best settings on `self` and returns their MSE.
    fn gpu_optimize_settings(&mut self, ctx: &GpuContext, reference: &Spectrum) -> Result<f64>;
}

impl GpuDeconvoluter for Deconvoluter {
    fn gpu_deconvolute_spectrum(&self, ctx: &GpuContext, spectrum: &Spectrum) -> Result<Deconvolution> {
        let settings = Settings::of(self);
        let s = settings.to_ffi(ctx.options())?;
        let ig = ignore_pairs(self);
        let (sb0, sb1) = spectrum.signal_boundaries(); // ordered as stored (spectrum.rs:854-863)
        let (x, y) = (spectrum.chemical_shifts(), spectrum.intensities());
        let mut cap = 4096usize;
        loop {
            let mut out = vec![ffi::MdgLorentzian::default(); cap];
            let (mut count, mut mse) = (0usize, 0f64);
            let st = unsafe {
                ffi::mdg_deconvolute(
                    ctx.raw(),
                    x.as_ptr(),
                    y.as_ptr(),
                    y.len(),
                    sb0,
                    sb1,
                    &s,
                    opt_ptr(&ig),
                    ig.len() / 2,
                    out.as_mut_ptr(),
                    cap,
                    &mut count,
                    &mut mse,
                )
            };
            match st {
                ffi::MDG_OK => return Ok(settings.deconvolution(&out[..count], mse)),
                ffi::MDG_CAPACITY if count > cap => cap = count, // two-phase size query
                _ => return Err(settings.error(st)),
            }
        }
    }

    fn gpu_deconvolute_spectra<S: AsRef<Spectrum>>(
        &self,
        ctx: &GpuContext,
        spectra: &[S],
    ) -> Result<Vec<Deconvolution>> {
        let settings = Settings::of(self);
        let s = settings.to_ffi(ctx.options())?;
        let ig = ignore_pairs(self);
        let mut results: Vec<Option<(c_int, Vec<ffi::MdgLorentzian>, f64)>> =
            (0..spectra.len()).map(|_| None).collect();
        let mut lengths: Vec<usize> = spectra.iter().map(|sp| sp.as_ref().len()).collect();
        lengths.sort_unstable();
        lengths.dedup();
        for n in lengths {
            let idx: Vec<usize> = (0..spectra.len())
                .filter(|&i| spectra[i].as_ref().len() == n)
                .collect();
            let b = idx.len();
            // the spectra's own rows (Arc<[f64]>, spectrum.rs:101-105), no stacking copy;
            // spectra sharing one axis Arc pass one pointer, uploaded once
            let (mut x, mut y, mut sb) = (Vec::with_capacity(b), Vec::with_capacity(b), Vec::new());
            for &i in &idx {
                let sp = spectra[i].as_ref();
                x.push(sp.chemical_shifts().as_ptr());
                y.push(sp.intensities().as_ptr());
                let (a, c) = sp.signal_boundaries();
                sb.extend_from_slice(&[a, c]);
            }
            let cap = n / 2 + 2; // the engine's peak capacity bound
            let mut out = vec![ffi::MdgLorentzian::default(); b * cap];
            let mut counts = vec![0usize; b];
            let mut mse = vec![0f64; b];
            let mut status = vec![0 as c_int; b];
            let rc = unsafe {
                ffi::mdg_deconvolute_rows(
                    ctx.raw(),
                    b,
                    n,
                    x.as_ptr(),
                    y.as_ptr(),
                    sb.as_ptr(),
                    &s,
                    opt_ptr(&ig),
                    ig.len() / 2,
                    out.as_mut_ptr(),
                    cap,
                    counts.as_mut_ptr(),
                    mse.as_mut_ptr(),
                    status.as_mut_ptr(),
                )
            };
            if rc >= 100 || rc == ffi::MDG_INVALID_ARGUMENT {
                return Err(engine_error(rc));
            }
            for (k, &i) in idx.iter().enumerate() {
                let rows = out[k * cap..k * cap + counts[k].min(cap)].to_vec();
                results[i] = Some((status[k], rows, mse[k]));
            }
        }
        results
            .into_iter()
            .map(|r| {
                let (st, rows, mse) = r.expect("every spectrum ran");
                if st == ffi::MDG_OK {
                    Ok(settings.deconvolution(&rows, mse))
                } else {
                    Err(settings.error(st))
                }
            })
            .collect()
    }

    fn gpu_optimize_settings(&mut self, ctx: &GpuContext, reference: &Spectrum) -> Result<f64> {
        let settings = Settings::of(self);
        let ig = ignore_pairs(self);
        let (sb0, sb1) = reference.signal_boundaries();
        let mut best = ffi::MdgSettings::default();
        let mut mse = 0f64;
        let st = unsafe {
            ffi::mdg_optimize_settings(
                ctx.raw(),
                reference.chemical_shifts().as_ptr(),
                reference.intensities().as_ptr(),
                reference.len(),
                sb0,
                sb1,
                opt_ptr(&ig),
                ig.len() / 2,
                &mut best,
                &mut mse,
            )
        };
        if st != ffi::MDG_OK {
            return Err(settings.error(st));
        }
        self.set_smoothing_settings(SmoothingSettings::MovingAverage {
            iterations: best.smooth_iterations as usize,
            window_size: best.smooth_window as usize,
        })?;
        self.set_selection_settings(SelectionSettings::NoiseScoreFilter {
            scoring_method: ScoringMethod::MinimumSum,
            threshold: best.threshold,
        })?;
        self.set_fitting_settings(FittingSettings::Analytical {
            iterations: best.fit_iterations as usize,
        })?;
        Ok(mse)
    }
}

/// `Lorentzian::superposition_vec` / `par_superposition_vec` (lorentzian.rs:631-663):
/// every point's sum in slice order, bit-identical to the reference.
pub fn gpu_superposition_vec<L: AsRef<Lorentzian>>(
    ctx: &GpuContext,
    x: &[f64],
    lorentzians: &[L],
) -> Result<Vec<f64>> {
    let params: Vec<ffi::MdgLorentzian> = lorentzians
        .iter()
        .map(|l| {
            let l = l.as_ref();
            ffi::MdgLorentzian {
                sfhw: l.sfhw(),
                hw2: l.hw2(),
                maxp: l.maxp(),
            }
        })
        .collect();
    let mut out = vec![0f64; x.len()];
    check(unsafe {
        ffi::mdg_superposition_vec(
            ctx.raw(),
            x.as_ptr(),
            x.len(),
            params.as_ptr(),
            params.len(),
            out.as_mut_ptr(),
        )
    })?;
    Ok(out)
}

/// One JCAMP-DX data block (the text after `##XYDATA=` / `##DATA TABLE=`, trimmed)
/// decoded natively into intensities times `factor`, as `JcampDx::decode_asdf` /
/// `decode_affn` do (spectrum/formats/jcampdx.rs:892-1091). `None` when the native
/// decoder leaves the block to the reader's own decode (non-ASCII text, or data the
/// reference rejects, which the reader's decode then reports with its own error).
/// Host only: no GPU is touched.
pub fn jcampdx_decode(block: &str, factor: f64) -> Result<Option<Vec<f64>>> {
    // a first guess; DUP counts can expand a short token into many values, so a block
    // that needs more reports its count with MDG_CAPACITY (nothing written) and is
    // decoded again into a buffer of that size
    let mut out = vec![0f64; block.len() + 1];
    loop {
        let mut n = 0usize;
        let rc = unsafe {
            ffi::mdg_jcampdx_decode(
                block.as_ptr() as *const c_char,
                block.len(),
                factor,
                out.as_mut_ptr(),
                out.len(),
                &mut n,
            )
        };
        match rc {
            ffi::MDG_INVALID_ARGUMENT => return Ok(None),
            ffi::MDG_CAPACITY if n > out.len() => out.resize(n, 0.0),
            _ => {
                check(rc)?;
                out.truncate(n);
                return Ok(Some(out));
            }
        }
    }
}

/// ABI version of the loaded library (mdgpu.h `MDG_ABI_VERSION`).
pub fn abi_version() -> i32 {
    unsafe { ffi::mdg_abi_version() }
}
