//go:build hip

// Package ocl, HIP build: the MI355X drop-in for internal/ocl/ocltracer.go.
//
// Copy this file to internal/ocl/ocltracer_hip.go of pathtracer-ocl, put
// `//go:build !hip` on the first line of ocltracer.go, and place libptmi.so and
// include/ptmi.h under third_party/ptmi/{lib,include} (or change the two #cgo lines).
// `go build -tags hip ./cmd/pt` then renders through libptmi.so; without the tag the
// OpenCL path is built exactly as before.  Nothing else in the Go program changes:
// BuildSceneBufferCL, the camera, OBJ/BVH loading and the PNG/.raw output stay as they are.
//
// tests/go_abi/go_sequence.c makes the same C calls, with the same arguments in the
// same order, and is run on the GPU by tests/test_gpu_go_abi.py (this image has no Go
// toolchain, so this file itself has not been compiled here).
package ocl

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/ptmi/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/ptmi/lib -lptmi -Wl,-rpath,${SRCDIR}/../../third_party/ptmi/lib
#include <stdlib.h>
#include "ptmi.h"
*/
import "C"

import (
	"fmt"
	"image"
	"image/draw"
	"math/rand"
	"unsafe"

	"github.com/sirupsen/logrus"
)

func init() {
	// The C side reads the records at the reference's fixed sizes (ocltracer.go:25-96).
	if unsafe.Sizeof(CLObject{}) != C.PTMI_OBJECT_BYTES || unsafe.Sizeof(CLTriangle{}) != C.PTMI_TRIANGLE_BYTES ||
		unsafe.Sizeof(CLGroup{}) != C.PTMI_GROUP_BYTES || unsafe.Sizeof(CLCamera{}) != C.PTMI_CAMERA_BYTES {
		panic("ocl: record sizes do not match ptmi.h")
	}
}

// frameSeeds draws one rand.Float64() per pixel, as computeBatch does (ocltracer.go:260-263).
func frameSeeds(camera CLCamera) []float64 {
	seeds := make([]float64, int(camera.Width)*int(camera.Height))
	for i := range seeds {
		seeds[i] = rand.Float64()
	}
	return seeds
}

// records returns &slice[0] of each record slice (nil for an empty one). The records
// hold no Go pointers, so passing them to C is legal under the cgo pointer rules.
func records(objects []CLObject, triangles []CLTriangle, groups []CLGroup) (obj, tris, grps unsafe.Pointer) {
	if len(objects) > 0 {
		obj = unsafe.Pointer(&objects[0])
	}
	if len(triangles) > 0 {
		tris = unsafe.Pointer(&triangles[0])
	}
	if len(groups) > 0 {
		grps = unsafe.Pointer(&groups[0])
	}
	return
}

// textureArrays packs the three image lists as prepareTextures does (ocltracer.go:228-254)
// into C memory (freed by the returned func), so the struct holds no Go pointers.
func textureArrays(textures, sphereTextures, cubeTextures []image.Image) (C.ptmi_textures, func()) {
	var tex C.ptmi_textures
	var blocks []unsafe.Pointer
	for k, list := range [][]image.Image{textures, sphereTextures, cubeTextures} {
		if len(list) == 0 {
			continue // the reference's all-zero fake image
		}
		b := list[0].Bounds()
		need := b.Dx() * b.Dy() * 4 * len(list)
		all := make([]byte, 0, need)
		for _, img := range list {
			nrgba, ok := img.(*image.NRGBA)
			if !ok { // LoadImage already returns NRGBA; convert anything else the same way
				nrgba = image.NewNRGBA(img.Bounds())
				draw.Draw(nrgba, nrgba.Bounds(), img, img.Bounds().Min, draw.Src)
			}
			all = append(all, nrgba.Pix...)
		}
		if len(all) < need {
			all = append(all, make([]byte, need-len(all))...)
		}
		p := C.CBytes(all[:need])
		blocks = append(blocks, p)
		tex.pixels[k] = (*C.uint8_t)(p)
		tex.width[k], tex.height[k], tex.count[k] = C.uint32_t(b.Dx()), C.uint32_t(b.Dy()), C.uint32_t(len(list))
	}
	return tex, func() {
		for _, p := range blocks {
			C.free(p)
		}
	}
}

// Trace has the signature and contract of the OpenCL version (ocltracer.go:98-100):
// float64 RGBA, W*H*4 values, RGB = sum of samples / samples, A = 1.
func Trace(objects []CLObject, triangles []CLTriangle, groups []CLGroup, deviceIndex, samples int,
	camera CLCamera, textures []image.Image, sphereTextures []image.Image, cubeTextures []image.Image) []float64 {
	logrus.Infof("trace with %d objects %dx%d (ptmi/HIP)", len(objects), camera.Width, camera.Height)
	seeds := frameSeeds(camera)
	out := make([]float64, len(seeds)*4)
	obj, tris, grps := records(objects, triangles, groups)
	tex, free := textureArrays(textures, sphereTextures, cubeTextures)
	defer free()
	var errBuf [512]C.char
	rc := C.ptmi_trace(obj, C.uint32_t(len(objects)), tris, C.uint32_t(len(triangles)),
		grps, C.uint32_t(len(groups)), C.int(deviceIndex), C.uint32_t(samples), unsafe.Pointer(&camera),
		(*C.double)(unsafe.Pointer(&seeds[0])), 0, &tex, (*C.double)(unsafe.Pointer(&out[0])),
		&errBuf[0], C.size_t(len(errBuf)))
	if rc != C.PTMI_OK {
		// The reference treats every driver failure as fatal (ocltracer.go:124-174).
		logrus.Fatalf("ptmi_trace failed (%d): %s", int(rc), C.GoString(&errBuf[0]))
	}
	return out
}

// TraceMulti renders one frame over several GPUs of this process (ptmi_trace_multi):
// split "sample" gives every device a cost-balanced range of sample indices of every
// pixel, "tile" the 8x8 tiles t with t % len(devices) == d; the partial frames are
// combined on devices[0] over xGMI. Same records, seeds and result as Trace. Backs a
// `--gpus N` flag of cmd/pt (main.go:47-56): devices 0..N-1.
func TraceMulti(objects []CLObject, triangles []CLTriangle, groups []CLGroup, devices []int, split string,
	samples int, camera CLCamera, textures []image.Image, sphereTextures []image.Image,
	cubeTextures []image.Image) []float64 {
	logrus.Infof("trace with %d objects %dx%d on %d GPUs, %s split (ptmi/HIP)", len(objects), camera.Width,
		camera.Height, len(devices), split)
	if len(devices) == 0 {
		logrus.Fatalf("TraceMulti: no devices")
	}
	mode := 0
	switch split {
	case "sample":
	case "tile":
		mode = 1
	default:
		logrus.Fatalf("TraceMulti: split must be \"sample\" or \"tile\", got %q", split)
	}
	devs := C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(C.int(0))))
	defer C.free(devs)
	for i, d := range devices {
		*(*C.int)(unsafe.Pointer(uintptr(devs) + uintptr(i)*unsafe.Sizeof(C.int(0)))) = C.int(d)
	}
	seeds := frameSeeds(camera)
	out := make([]float64, len(seeds)*4)
	obj, tris, grps := records(objects, triangles, groups)
	tex, free := textureArrays(textures, sphereTextures, cubeTextures)
	defer free()
	var errBuf [512]C.char
	rc := C.ptmi_trace_multi(obj, C.uint32_t(len(objects)), tris, C.uint32_t(len(triangles)),
		grps, C.uint32_t(len(groups)), (*C.int)(devs), C.uint32_t(len(devices)), C.int(mode),
		C.uint32_t(samples), unsafe.Pointer(&camera), (*C.double)(unsafe.Pointer(&seeds[0])), 0, &tex,
		(*C.double)(unsafe.Pointer(&out[0])), &errBuf[0], C.size_t(len(errBuf)))
	if rc != C.PTMI_OK {
		logrus.Fatalf("ptmi_trace_multi failed (%d): %s", int(rc), C.GoString(&errBuf[0]))
	}
	return out
}

// DeviceCount is the number of HIP devices ptmi can use.
func DeviceCount() int { return int(C.ptmi_device_count()) }

// ListDevices backs --list-devices (cmd/pt/main.go:98-112) without OpenCL.
func ListDevices() {
	var name [256]C.char
	for i := 0; i < DeviceCount(); i++ {
		C.ptmi_device_name(C.int(i), &name[0], C.size_t(len(name)))
		fmt.Printf("Index: %d Type: GPU Name: %s\n", i, C.GoString(&name[0]))
	}
}
