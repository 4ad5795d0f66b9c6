//go:build amdgpu

// Package webp: the MI355X decode path behind the reference's public API.
//
// Drop this file into the reference's root package (github.com/DaanV2/go-webp, package
// webp) and build with `-tags amdgpu`.  It replaces the two stubs of decode.go:8-14
// (`Decode` / `DecodeConfig`, both panic("unimplemented") today) with calls into
// libgowebp_amd.so through the C ABI of include/gowebp_amd.h, and adds batch, multi-GPU and
// animation entry points.  The library keeps no Go pointer after a call returns (cgo rule):
// it copies inputs into its own pinned staging and writes outputs before returning.
//
// Layout assumed by the #cgo lines: the header under third_party/gowebp_amd/include and the
// library under third_party/gowebp_amd/lib, next to this file.  Neither this image nor the
// MI355X box has a Go toolchain (probed: profiles/r04/box_env_probe.txt), so the file is not
// compiled here; every C entry point it calls is exercised through the same ABI by tests/
// (ctypes), and tests/test_capi.py checks that each one it names is declared and exported.
package webp

/*
#cgo CFLAGS: -I${SRCDIR}/third_party/gowebp_amd/include
#cgo LDFLAGS: -L${SRCDIR}/third_party/gowebp_amd/lib -lgowebp_amd -Wl,-rpath,${SRCDIR}/third_party/gowebp_amd/lib
#include <stdlib.h>
#include "gowebp_amd.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"image"
	"image/color"
	"io"
	"runtime"
	"unsafe"
)

// VP8StatusCode names (pkg/vp8/enums.go:20-31), identical to wg_status.
var statusText = [...]string{"OK", "OUT_OF_MEMORY", "INVALID_PARAM", "BITSTREAM_ERROR",
	"UNSUPPORTED_FEATURE", "SUSPENDED", "USER_ABORT", "NOT_ENOUGH_DATA"}

// StatusError carries the VP8StatusCode of a failed decode.
type StatusError struct {
	Code int
	What string
}

func (e *StatusError) Error() string {
	name := "UNKNOWN"
	if e.Code >= 0 && e.Code < len(statusText) {
		name = statusText[e.Code]
	}
	return fmt.Sprintf("webp: %s: %s", e.What, name)
}

func statusErr(st C.int, what string) error {
	if st == C.WG_STATUS_OK {
		return nil
	}
	return &StatusError{Code: int(st), What: what}
}

// cBytes: a Go byte slice passed for the duration of one call (cgo pointer rule).  An empty
// slice is passed as NULL, which the library reports as INVALID_PARAM (as WebPDecode does for
// a NULL input) instead of indexing data[0].
func cBytes(data []byte) (*C.uint8_t, C.size_t) {
	if len(data) == 0 {
		return nil, 0
	}
	return (*C.uint8_t)(unsafe.Pointer(&data[0])), C.size_t(len(data))
}

// DecodeConfig replaces decode.go:12-14 (WebPGetFeatures, host only, no GPU needed).
func DecodeConfig(r io.Reader) (image.Config, error) {
	data, err := io.ReadAll(r)
	if err != nil {
		return image.Config{}, err
	}
	return decodeConfig(data)
}

func decodeConfig(data []byte) (image.Config, error) {
	if len(data) == 0 {
		return image.Config{}, &StatusError{Code: int(C.WG_STATUS_NOT_ENOUGH_DATA), What: "DecodeConfig"}
	}
	var f C.wg_features
	p, n := cBytes(data)
	if err := statusErr(C.wg_get_features(p, n, &f), "DecodeConfig"); err != nil {
		return image.Config{}, err
	}
	return image.Config{ColorModel: color.NRGBAModel, Width: int(f.width), Height: int(f.height)}, nil
}

// Decode replaces decode.go:8-10: one frame (lossy, lossless or lossy + ALPH) through the GPU
// path into an *image.NRGBA (opaque lossy input => A = 255).  The device is the one chosen by
// SetDevice (0 by default).
func Decode(r io.Reader) (image.Image, error) {
	data, err := io.ReadAll(r)
	if err != nil {
		return nil, err
	}
	cfg, err := decodeConfig(data)
	if err != nil {
		return nil, err
	}
	img := image.NewNRGBA(image.Rect(0, 0, cfg.Width, cfg.Height))
	p, n := cBytes(data)
	st := C.wg_decode_rgba_into(p, n, (*C.uint8_t)(unsafe.Pointer(&img.Pix[0])), C.size_t(len(img.Pix)),
		C.int(img.Stride), 0)
	if err := statusErr(st, "Decode"); err != nil {
		return nil, err
	}
	return img, nil
}

// YUVA holds the planes of a MODE_YUV / MODE_YUVA decode (WebPYUVABuffer, buffer.go:17-25): Y
// (W x H), U and V ((W+1)/2 x (H+1)/2) and, with alpha requested, A (W x H; 0xff for frames
// without ALPH).  The samples are VP8's (studio-swing BT.601), not image.YCbCr's JFIF ones, so
// they are returned as planes rather than as an image.YCbCr whose At() would convert them with
// the wrong matrix.
type YUVA struct {
	W, H                       int
	Y, U, V, A                 []byte
	YStride, UVStride, AStride int
}

// DecodeYUVA decodes one frame to its Y / U / V (/ A) planes on the GPU (wg_decode_yuv_into:
// WebPDecode with config.output.colorspace MODE_YUV = 11 or MODE_YUVA = 12, webp.go:870-909).
// Lossy frames give their reconstructed planes; lossless ones libwebp 1.6.0's ARGB -> YUV(A)
// conversion.
func DecodeYUVA(r io.Reader, withAlpha bool) (*YUVA, error) {
	data, err := io.ReadAll(r)
	if err != nil {
		return nil, err
	}
	cfg, err := decodeConfig(data)
	if err != nil {
		return nil, err
	}
	w, h := cfg.Width, cfg.Height
	uw, uh := (w+1)/2, (h+1)/2
	out := &YUVA{W: w, H: h, Y: make([]byte, w*h), U: make([]byte, uw*uh), V: make([]byte, uw*uh),
		YStride: w, UVStride: uw}
	var opt C.wg_decoder_options
	opt.colorspace = 11
	var buf C.wg_yuva_buffer
	// (Go memory for the duration of the call: pinned, the struct holding its pointers is C's)
	var pin runtime.Pinner
	defer pin.Unpin()
	pin.Pin(&out.Y[0])
	pin.Pin(&out.U[0])
	pin.Pin(&out.V[0])
	buf.y = (*C.uint8_t)(unsafe.Pointer(&out.Y[0]))
	buf.u = (*C.uint8_t)(unsafe.Pointer(&out.U[0]))
	buf.v = (*C.uint8_t)(unsafe.Pointer(&out.V[0]))
	buf.y_stride, buf.u_stride, buf.v_stride = C.int32_t(w), C.int32_t(uw), C.int32_t(uw)
	buf.y_size, buf.u_size, buf.v_size = C.size_t(len(out.Y)), C.size_t(len(out.U)), C.size_t(len(out.V))
	if withAlpha {
		opt.colorspace = 12
		out.A, out.AStride = make([]byte, w*h), w
		pin.Pin(&out.A[0])
		buf.a, buf.a_stride, buf.a_size = (*C.uint8_t)(unsafe.Pointer(&out.A[0])), C.int32_t(w), C.size_t(len(out.A))
	}
	cbuf := (*C.wg_yuva_buffer)(C.malloc(C.size_t(unsafe.Sizeof(buf))))
	defer C.free(unsafe.Pointer(cbuf))
	*cbuf = buf
	copt := (*C.wg_decoder_options)(C.malloc(C.size_t(unsafe.Sizeof(opt))))
	defer C.free(unsafe.Pointer(copt))
	*copt = opt
	p, n := cBytes(data)
	if err := statusErr(C.wg_decode_yuv_into(p, n, copt, cbuf), "DecodeYUVA"); err != nil {
		return nil, err
	}
	return out, nil
}

// SetDevice selects the HIP device behind Decode (wg_set_default_device).
func SetDevice(device int) error {
	return statusErr(C.wg_set_default_device(C.int(device)), "SetDevice")
}

// Decoder is one device context (wg_ctx): reuse it for batches.  Its pinned staging, worker
// pool and device buffers are kept between calls and released by Close.
type Decoder struct{ ctx *C.wg_ctx }

func NewDecoder(device, hostThreads int) (*Decoder, error) {
	c := C.wg_ctx_create(C.int(device), C.int(hostThreads))
	if c == nil {
		return nil, errors.New("webp: no usable HIP device")
	}
	return &Decoder{ctx: c}, nil
}

func (d *Decoder) Close() {
	if d.ctx != nil {
		C.wg_ctx_destroy(d.ctx)
		d.ctx = nil
	}
}

// batchArgs: C-allocated pointer tables for a batch call (Go memory may not hold Go pointers
// across the call) with inputs and outputs pinned until free().
type batchArgs struct {
	n               int
	dataP, outP     []*C.uint8_t
	sizes, caps     []C.size_t
	strides, status []C.int32_t
	raw             []unsafe.Pointer
	pinner          runtime.Pinner
	imgs            []*image.NRGBA
	errs            []error
}

func cAlloc[T any](a *batchArgs, n int) []T {
	var z T
	p := C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(z)))
	a.raw = append(a.raw, p)
	return unsafe.Slice((*T)(p), n)
}

func newBatchArgs(frames [][]byte) *batchArgs {
	n := len(frames)
	a := &batchArgs{n: n, imgs: make([]*image.NRGBA, n), errs: make([]error, n)}
	a.dataP = cAlloc[*C.uint8_t](a, n)
	a.outP = cAlloc[*C.uint8_t](a, n)
	a.sizes = cAlloc[C.size_t](a, n)
	a.caps = cAlloc[C.size_t](a, n)
	a.strides = cAlloc[C.int32_t](a, n)
	a.status = cAlloc[C.int32_t](a, n)
	for i, f := range frames {
		cfg, err := decodeConfig(f)
		if err != nil {
			a.errs[i] = err
			cfg = image.Config{Width: 1, Height: 1}
		}
		a.imgs[i] = image.NewNRGBA(image.Rect(0, 0, cfg.Width, cfg.Height))
		if len(f) > 0 { // an empty frame gets a per-frame status, it is not pinned or indexed
			a.pinner.Pin(&f[0])
		}
		a.pinner.Pin(&a.imgs[i].Pix[0])
		a.dataP[i], a.sizes[i] = cBytes(f)
		a.outP[i] = (*C.uint8_t)(unsafe.Pointer(&a.imgs[i].Pix[0]))
		a.strides[i] = C.int32_t(a.imgs[i].Stride)
		a.caps[i] = C.size_t(len(a.imgs[i].Pix))
	}
	return a
}

func (a *batchArgs) finish(st C.int, what string) ([]*image.NRGBA, []error) {
	defer a.free()
	if err := statusErr(st, what); err != nil {
		for i := range a.errs {
			a.errs[i] = err
		}
		return nil, a.errs
	}
	for i := 0; i < a.n; i++ {
		if a.errs[i] == nil {
			a.errs[i] = statusErr(C.int(a.status[i]), fmt.Sprintf("frame %d", i))
		}
		if a.errs[i] != nil {
			a.imgs[i] = nil
		}
	}
	return a.imgs, a.errs
}

func (a *batchArgs) free() {
	a.pinner.Unpin()
	for _, p := range a.raw {
		C.free(p)
	}
	a.raw = nil
}

// DecodeBatch decodes independent frames (entropy stage on the context's host threads, the DSP
// kernels on the device, pipelined in chunks: wg_decode_rgba_batch).  Per-frame errors do not
// abort the batch.
func (d *Decoder) DecodeBatch(frames [][]byte) ([]*image.NRGBA, []error) {
	if len(frames) == 0 {
		return nil, nil
	}
	a := newBatchArgs(frames)
	st := C.wg_decode_rgba_batch(d.ctx, &a.dataP[0], &a.sizes[0], C.int(a.n), &a.outP[0], &a.strides[0],
		&a.caps[0], &a.status[0], 0)
	return a.finish(st, "DecodeBatch")
}

// SetChunkFrames sets the pipeline chunk of DecodeBatch (wg_ctx_set_chunk_frames; 0 = automatic).
func (d *Decoder) SetChunkFrames(frames int) error {
	return statusErr(C.wg_ctx_set_chunk_frames(d.ctx, C.int(frames)), "SetChunkFrames")
}

// Stats: where the last DecodeBatch's time went (wg_ctx_pipeline_stats).
func (d *Decoder) Stats() (C.wg_pipeline_stats, error) {
	var ps C.wg_pipeline_stats
	err := statusErr(C.wg_ctx_pipeline_stats(d.ctx, &ps), "Stats")
	return ps, err
}

// PinnedNRGBA is an *image.NRGBA whose Pix lives in page-locked C memory (wg_host_alloc): the
// device writes it by DMA.  Being C memory it needs no runtime.Pinner; release it with Free.
type PinnedNRGBA struct {
	*image.NRGBA
	p     unsafe.Pointer
	bytes int // size of the C block at p (the capacity the library checks every frame against)
}

func NewPinnedNRGBA(w, h int) (*PinnedNRGBA, error) {
	p := C.wg_host_alloc(C.size_t(4 * w * h))
	if p == nil {
		return nil, &StatusError{Code: int(C.WG_STATUS_OUT_OF_MEMORY), What: "NewPinnedNRGBA"}
	}
	pix := unsafe.Slice((*byte)(p), 4*w*h)
	return &PinnedNRGBA{NRGBA: &image.NRGBA{Pix: pix, Stride: 4 * w, Rect: image.Rect(0, 0, w, h)}, p: p,
		bytes: 4 * w * h}, nil
}

func (m *PinnedNRGBA) Free() {
	if m.p != nil {
		C.wg_host_free(m.p)
		m.p, m.NRGBA, m.bytes = nil, nil, 0
	}
}

// DecodeBatchInto decodes frames[i] into dst[i] (reused across calls, e.g. PinnedNRGBA
// buffers of a serving loop); dst[i] must hold frame i (Stride >= 4 * width, enough rows).
// Per-frame errors: a nil or freed dst[i] is INVALID_PARAM here, and the library checks every
// frame's window against dst[i]'s allocation (INVALID_PARAM, nothing written) -- a frame larger
// than the buffer reused for it never writes past the buffer.
func (d *Decoder) DecodeBatchInto(frames [][]byte, dst []*PinnedNRGBA) []error {
	n := len(frames)
	errs := make([]error, n)
	if n == 0 || len(dst) != n {
		return errs
	}
	a := &batchArgs{n: n}
	defer a.free()
	a.dataP = cAlloc[*C.uint8_t](a, n)
	a.outP = cAlloc[*C.uint8_t](a, n)
	a.sizes = cAlloc[C.size_t](a, n)
	a.caps = cAlloc[C.size_t](a, n)
	a.strides = cAlloc[C.int32_t](a, n)
	a.status = cAlloc[C.int32_t](a, n)
	for i, f := range frames {
		if len(f) > 0 {
			a.pinner.Pin(&f[0])
		}
		a.dataP[i], a.sizes[i] = cBytes(f)
		if dst[i] == nil || dst[i].p == nil || dst[i].NRGBA == nil {
			// NULL output: the library reports INVALID_PARAM for the frame
			errs[i] = &StatusError{Code: int(C.WG_STATUS_INVALID_PARAM), What: fmt.Sprintf("frame %d: no buffer", i)}
			continue
		}
		a.outP[i] = (*C.uint8_t)(dst[i].p) // C memory: no pinning needed
		a.strides[i] = C.int32_t(dst[i].Stride)
		a.caps[i] = C.size_t(dst[i].bytes)
	}
	st := C.wg_decode_rgba_batch(d.ctx, &a.dataP[0], &a.sizes[0], C.int(n), &a.outP[0], &a.strides[0],
		&a.caps[0], &a.status[0], 0)
	for i := range errs {
		if errs[i] != nil {
			continue
		}
		if err := statusErr(st, "DecodeBatchInto"); err != nil {
			errs[i] = err
		} else {
			errs[i] = statusErr(C.int(a.status[i]), fmt.Sprintf("frame %d", i))
		}
	}
	return errs
}

// MultiDecoder shards frames across several contexts, normally one per GPU (SURVEY §8(e)):
// frames are independent, nothing is exchanged between devices.
type MultiDecoder struct{ ctxs []*C.wg_ctx }

func NewMultiDecoder(devices []int, hostThreadsPerDevice int) (*MultiDecoder, error) {
	m := &MultiDecoder{}
	for _, dev := range devices {
		c := C.wg_ctx_create(C.int(dev), C.int(hostThreadsPerDevice))
		if c == nil {
			m.Close()
			return nil, fmt.Errorf("webp: HIP device %d not usable", dev)
		}
		m.ctxs = append(m.ctxs, c)
	}
	return m, nil
}

func (m *MultiDecoder) Close() {
	for _, c := range m.ctxs {
		C.wg_ctx_destroy(c)
	}
	m.ctxs = nil
}

// DecodeBatch: contiguous shards of `frames`, one per device, decoded concurrently
// (wg_decode_rgba_batch_multi); results in input order.
func (m *MultiDecoder) DecodeBatch(frames [][]byte) ([]*image.NRGBA, []error) {
	if len(frames) == 0 || len(m.ctxs) == 0 {
		return nil, nil
	}
	a := newBatchArgs(frames)
	ctxs := cAlloc[*C.wg_ctx](a, len(m.ctxs))
	copy(ctxs, m.ctxs)
	st := C.wg_decode_rgba_batch_multi(&ctxs[0], C.int(len(ctxs)), &a.dataP[0], &a.sizes[0], C.int(a.n), &a.outP[0],
		&a.strides[0], &a.caps[0], &a.status[0], 0)
	return a.finish(st, "MultiDecoder.DecodeBatch")
}

// DecodeAnimation: every canvas of an animated WebP (WebPAnimDecoder's GetNext loop) as
// *image.NRGBA frames plus end timestamps in ms.
func (d *Decoder) DecodeAnimation(data []byte) ([]*image.NRGBA, []int, error) {
	if len(data) == 0 {
		return nil, nil, &StatusError{Code: int(C.WG_STATUS_NOT_ENOUGH_DATA), What: "DecodeAnimation"}
	}
	var info C.wg_anim_info
	p, n := cBytes(data)
	if err := statusErr(C.wg_anim_demux(p, n, &info, nil, 0), "DecodeAnimation"); err != nil {
		return nil, nil, err
	}
	w, h, f := int(info.canvas_width), int(info.canvas_height), int(info.frame_count)
	if f == 0 || w == 0 || h == 0 {
		return nil, nil, nil
	}
	canvases := make([]byte, f*w*h*4)
	ts := make([]int32, f)
	var pinner runtime.Pinner
	defer pinner.Unpin()
	pinner.Pin(&data[0])
	pinner.Pin(&canvases[0])
	pinner.Pin(&ts[0])
	st := C.wg_anim_decode(d.ctx, p, n, (*C.uint8_t)(unsafe.Pointer(&canvases[0])),
		(*C.int32_t)(unsafe.Pointer(&ts[0])), 0)
	if err := statusErr(st, "DecodeAnimation"); err != nil {
		return nil, nil, err
	}
	frames := make([]*image.NRGBA, f)
	times := make([]int, f)
	for i := range frames {
		frames[i] = &image.NRGBA{Pix: canvases[i*w*h*4 : (i+1)*w*h*4], Stride: 4 * w,
			Rect: image.Rect(0, 0, w, h)}
		times[i] = int(ts[i])
	}
	return frames, times, nil
}

func init() {
	// image.Decode registration (the reference has none yet): "RIFF????WEBPVP8"
	image.RegisterFormat("webp", "RIFF????WEBPVP8", Decode, DecodeConfig)
}
