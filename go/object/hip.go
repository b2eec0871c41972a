//go:build cgo && honu_hip

// Package object: the gfx950 batch codec behind Honu's pkg/store/object API.
//
// STATUS: UNVERIFIED. Neither the build container nor the GPU box of this
// repository has a Go toolchain (profiles/r01_gpu_box_toolchains.txt), so this
// file has never been compiled. It is the cgo binding a maintainer vendors
// into rotationalio/honu's pkg/store/object (INTEGRATION.md), kept behind the
// `honu_hip` build tag so the pure-Go Marshal / Metadata / Data stay the
// default (the reference builds with CGO_ENABLED=0, Dockerfile:24). The C ABI
// it calls (include/honu_codec.h) is exercised on the GPU from plain C by
// honu_amd/c_abi_demo.c, which runs this file's MarshalBatch / DecodeBatch
// call sequence (tests/test_c_abi.py), and from Python by the test suite.
//
// Reference functions replaced, one batch per call instead of one record:
//
//	object.Marshal            object.go:24-45  -> (*Codec).MarshalBatch
//	(Object).Metadata / Data  object.go:66-99  -> (*Codec).DecodeBatch
package object

/*
#cgo CFLAGS: -I${SRCDIR}/internal/hip
#cgo LDFLAGS: -L${SRCDIR}/internal/hip -lhonu_codec -Wl,-rpath,${SRCDIR}/internal/hip
#include <stdlib.h>
#include "honu_codec.h"
*/
import "C"

import (
	"encoding/binary"
	"errors"
	"fmt"
	"io"
	"net"
	"time"
	"unsafe"

	"go.rtnl.ai/honu/pkg/region"
	"go.rtnl.ai/honu/pkg/store/lamport"
	"go.rtnl.ai/honu/pkg/store/lani"
	"go.rtnl.ai/honu/pkg/store/metadata"
	"go.rtnl.ai/ulid"
)

var ErrGoPanic = errors.New("object: input on which the pure-Go codec panics")
var ErrInput = errors.New("object: a row's span or list lies outside its arena")
var ErrCapacity = errors.New("object: GPU output arena or table too small")

var statusErr = map[C.int32_t]error{
	C.HONU_ERR_BAD_VERSION:    ErrBadVersion,
	C.HONU_ERR_MALFORMED:      ErrMalformed,
	C.HONU_ERR_EOF:            io.EOF,
	C.HONU_ERR_UNEXPECTED_EOF: io.ErrUnexpectedEOF,
	C.HONU_ERR_NO_LENGTH:      lani.ErrNoLength,
	C.HONU_ERR_PARSE_BOOLEAN:  lani.ErrParseBoolean,
	C.HONU_ERR_PARSE_VARINT:   lani.ErrParseVarInt,
	C.HONU_ERR_PANIC:          ErrGoPanic,
	C.HONU_ERR_INPUT:          ErrInput,
	C.HONU_ERR_CAPACITY:       ErrCapacity,
}

// recordErr maps a per-record status to an error; an unknown code is an
// error too, so no failed record can come back as (nil, nil).
func recordErr(st C.int32_t) error {
	if st == C.HONU_OK {
		return nil
	}
	if err, ok := statusErr[st]; ok {
		return err
	}
	return fmt.Errorf("object: unknown codec status %d", int32(st))
}

// call checks a call-level status (HONU_E_ARG, HONU_E_WORKSPACE, HONU_E_HIP, ...).
func call(what string, st C.int32_t) error {
	if st == C.HONU_OK {
		return nil
	}
	return fmt.Errorf("%s: %s (%s)", what, C.GoString(C.honu_status_string(st)),
		C.GoString(C.honu_last_error()))
}

// Codec owns one device context. Buffers handed to C live in C memory
// (pinned host / device), never in the Go heap, so asynchronous GPU work
// obeys the cgo pointer-passing rules.
type Codec struct {
	ctx    *C.honu_ctx
	stream unsafe.Pointer // nil: the null stream
	// ACL table entries / regions per record of the last decoded batch: the
	// first guess for the next batch's table sizes (DecodeBatch). With the
	// ACL lists returned in place (the default) only lists holding a nil
	// entry take table entries.
	aclPerRecord, regPerRecord uint64
}

func NewCodec(device int, maxRecords uint64) (*Codec, error) {
	if v := C.honu_abi_version(); v != C.HONU_ABI_VERSION {
		return nil, fmt.Errorf("object: libhonu_codec ABI %d, this binding %d", v, C.HONU_ABI_VERSION)
	}
	var st C.int32_t
	ctx := C.honu_ctx_create(C.int(device), C.uint64_t(maxRecords), &st)
	if ctx == nil {
		return nil, errors.New(C.GoString(C.honu_status_string(st)))
	}
	return &Codec{ctx: ctx, aclPerRecord: 1, regPerRecord: 8}, nil
}

func (c *Codec) Close() { C.honu_ctx_destroy(c.ctx) }

// Param / SetParam: the context's launch parameters (honu_ctx_set_param,
// honu_ctx_get_param). "speculate" 0 turns the single-launch decode's
// speculation off for a context that mostly sees malformed records; without
// it the context backs off by itself for 16 calls after a recovery
// ("speculate_backoff" reads the calls left, "recoveries" counts them).
// "acl_inplace" 0 returns every ACL list in the table (unflatten reads both).
func (c *Codec) SetParam(name string, v int64) error {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	if st := C.honu_ctx_set_param(c.ctx, cs, C.int64_t(v)); st != 0 {
		return errors.New(C.GoString(C.honu_last_error()))
	}
	return nil
}

func (c *Codec) Param(name string) (int64, error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var v C.int64_t
	if st := C.honu_ctx_get_param(c.ctx, cs, &v); st != 0 {
		return 0, errors.New(C.GoString(C.honu_last_error()))
	}
	return int64(v), nil
}

// hostBuf / devBuf: pinned host and device allocations owned by C.
type hostBuf struct {
	p unsafe.Pointer
	n uintptr
}
type devBuf struct {
	p unsafe.Pointer
	n uintptr
}

func pinned(n uintptr) hostBuf { return hostBuf{C.honu_host_alloc(C.uint64_t(n + 16)), n} }
func device(n uintptr) devBuf  { return devBuf{C.honu_device_alloc(C.uint64_t(n + 16)), n} }
func (h hostBuf) bytes() []byte { return unsafe.Slice((*byte)(h.p), h.n) }
func (h hostBuf) free()         { C.honu_host_free(h.p) }
func (d devBuf) free()          { C.honu_device_free(d.p) }

// batch: one flattened batch in pinned memory (the encode input of
// include/honu_codec.h: rows, var arena, ACL table, region table, CSR
// payload arena).
type batch struct {
	rows, vars, acls, regs, pay, payOff hostBuf
	n, nacl, nreg                       uint64
}

type devBatch struct{ rows, vars, acls, regs, pay, payOff devBuf }

func (b *batch) free() {
	for _, h := range []hostBuf{b.rows, b.vars, b.acls, b.regs, b.pay, b.payOff} {
		h.free()
	}
}

func (d *devBatch) free() {
	for _, x := range []devBuf{d.rows, d.vars, d.acls, d.regs, d.pay, d.payOff} {
		x.free()
	}
}

func (b *batch) upload(stream unsafe.Pointer) (*devBatch, error) {
	d := &devBatch{}
	for _, x := range []struct {
		h hostBuf
		d *devBuf
	}{{b.rows, &d.rows}, {b.vars, &d.vars}, {b.acls, &d.acls}, {b.regs, &d.regs}, {b.pay, &d.pay},
		{b.payOff, &d.payOff}} {
		*x.d = device(x.h.n)
		if x.d.p == nil {
			d.free()
			return nil, errors.New("object: device allocation failed")
		}
		if err := call("upload", C.honu_memcpy_h2d(x.d.p, x.h.p, C.uint64_t(x.h.n), stream)); err != nil {
			d.free()
			return nil, err
		}
	}
	return d, nil
}

func cULID(u ulid.ULID) (o [16]C.uint8_t) {
	for k := range o {
		o[k] = C.uint8_t(u[k])
	}
	return o
}

// nanos: lani.EncodeTime (lani/encode.go:201-206): 0 for the zero time.
func nanos(t time.Time) C.int64_t {
	if t.IsZero() {
		return 0
	}
	return C.int64_t(t.UnixNano())
}

// flatten writes one honu_meta row per *metadata.Metadata (presence bits from
// the nil pointers, ULIDs inline, strings and byte slices appended to the var
// arena as {off, len}, ACL entries and regions appended to their tables,
// times as UnixNano or 0), and the payloads as a CSR arena; mirrors
// honu_amd/metadata.py:pack_batch. A nil *Metadata leaves an all-zero row
// (no HONU_HAS_META): the encoder reports HONU_ERR_PANIC, where Marshal(nil,
// ...) panics (metadata.go:66).
func flatten(metas []*metadata.Metadata, datas [][]byte) *batch {
	n := uint64(len(metas))
	var nvar, nacl, nreg, npay uint64
	for i, m := range metas {
		npay += uint64(len(datas[i]))
		if m == nil {
			continue
		}
		nvar += uint64(len(m.MIME))
		if m.Schema != nil {
			nvar += uint64(len(m.Schema.Name))
		}
		if p := m.Publisher; p != nil {
			nvar += uint64(len(p.IPAddress) + len(p.UserAgent))
		}
		if e := m.Encryption; e != nil {
			nvar += uint64(len(e.PublicKeyID) + len(e.EncryptionKey) + len(e.HMACSecret) + len(e.Signature))
		}
		nacl += uint64(len(m.ACL))
		nreg += uint64(len(m.WriteRegions))
	}
	b := &batch{n: n, nacl: nacl, nreg: nreg,
		rows: pinned(uintptr(n) * uintptr(C.sizeof_honu_meta)), vars: pinned(uintptr(nvar)),
		acls: pinned(uintptr(nacl) * uintptr(C.sizeof_honu_acl)), regs: pinned(4 * uintptr(nreg)),
		pay: pinned(uintptr(npay)), payOff: pinned(8 * uintptr(n+1))}
	rows := unsafe.Slice((*C.honu_meta)(b.rows.p), n)
	vars, pay := b.vars.bytes(), b.pay.bytes()
	acls := unsafe.Slice((*C.honu_acl)(b.acls.p), nacl)
	regs := unsafe.Slice((*uint32)(b.regs.p), nreg)
	payOff := unsafe.Slice((*uint64)(b.payOff.p), n+1)
	var v, a, g, p uint64
	span := func(s []byte) C.honu_span {
		if len(s) == 0 { // nil and empty encode alike (lani/encode.go Encode)
			return C.honu_span{}
		}
		o := v
		v += uint64(copy(vars[v:], s))
		return C.honu_span{off: C.uint64_t(o), len: C.uint64_t(len(s))}
	}
	for i, m := range metas {
		payOff[i] = p
		p += uint64(copy(pay[p:], datas[i]))
		r := &rows[i]
		*r = C.honu_meta{}
		if m == nil {
			continue
		}
		pr := uint32(C.HONU_HAS_META)
		r.object_id, r.collection_id = cULID(m.ObjectID), cULID(m.CollectionID)
		if ver := m.Version; ver != nil {
			pr |= C.HONU_HAS_VERSION
			r.pid, r.vid, r.region = C.uint32_t(ver.Scalar.PID), C.uint64_t(ver.Scalar.VID), C.uint32_t(ver.Region)
			if ver.Parent != nil {
				pr |= C.HONU_HAS_PARENT
				r.parent_pid, r.parent_vid = C.uint32_t(ver.Parent.PID), C.uint64_t(ver.Parent.VID)
			}
			if ver.Tombstone {
				r.tombstone = 1
			}
			r.version_created = nanos(ver.Created)
		}
		if s := m.Schema; s != nil {
			pr |= C.HONU_HAS_SCHEMA
			r.schema_name = span([]byte(s.Name))
			r.schema_major, r.schema_minor, r.schema_patch = C.uint32_t(s.Major), C.uint32_t(s.Minor), C.uint32_t(s.Patch)
		}
		r.mime = span([]byte(m.MIME))
		r.owner, r.group = cULID(m.Owner), cULID(m.Group)
		r.permissions = C.uint8_t(m.Permissions)
		if len(m.ACL) > 0 {
			r.acl_off, r.acl_count = C.uint64_t(a), C.uint64_t(len(m.ACL))
			nb := uint64(0) // the list's encoded length, carried (HONU_ACL_SIZED): the size pass reads no entry
			for _, e := range m.ACL {
				acls[a] = C.honu_acl{}
				nb++ // a nil entry encodes as one 0x00 flag byte
				if e != nil {
					acls[a].client_id, acls[a].permissions, acls[a].present = cULID(e.ClientID), C.uint8_t(e.Permissions), 1
					nb += 17 // 01 | ClientID | Permissions (acls.go:26-39)
				}
				a++
			}
			r.acl_bytes = C.uint64_t(nb)
			pr |= C.HONU_ACL_SIZED
		}
		if len(m.WriteRegions) > 0 {
			r.regions_off, r.regions_count = C.uint64_t(g), C.uint64_t(len(m.WriteRegions))
			for _, x := range m.WriteRegions {
				regs[g] = uint32(x)
				g++
			}
		}
		if pub := m.Publisher; pub != nil {
			pr |= C.HONU_HAS_PUBLISHER
			r.publisher_id, r.client_id = cULID(pub.PublisherID), cULID(pub.ClientID)
			r.ip_address, r.user_agent = span(pub.IPAddress), span([]byte(pub.UserAgent))
		}
		if e := m.Encryption; e != nil {
			pr |= C.HONU_HAS_ENCRYPTION
			r.public_key_id, r.encryption_key = span([]byte(e.PublicKeyID)), span(e.EncryptionKey)
			r.hmac_secret, r.signature = span(e.HMACSecret), span(e.Signature)
			r.sealing_alg, r.encryption_alg = C.uint8_t(e.SealingAlgorithm), C.uint8_t(e.EncryptionAlgorithm)
			r.signature_alg = C.uint8_t(e.SignatureAlgorithm)
		}
		if cmp := m.Compression; cmp != nil {
			pr |= C.HONU_HAS_COMPRESSION
			r.compression_alg, r.compression_level = C.uint8_t(cmp.Algorithm), C.int64_t(cmp.Level)
		}
		r.flags = C.uint8_t(m.Flags)
		r.created, r.modified = nanos(m.Created), nanos(m.Modified)
		r.present = C.uint32_t(pr)
	}
	payOff[n] = p
	return b
}

// MarshalBatch is object.Marshal for many records in one GPU pass.
func (c *Codec) MarshalBatch(metas []*metadata.Metadata, datas [][]byte) ([]Object, []error, error) {
	n := len(metas)
	// 1. flatten into pinned C memory, 2. host -> device
	b := flatten(metas, datas)
	defer b.free()
	d, err := b.upload(c.stream)
	if err != nil {
		return nil, nil, err
	}
	defer d.free()
	// 3. sizes + exclusive scan -> output offsets; read the total back
	outOff, status, hOff := device(8*uintptr(n+1)), device(4*uintptr(n)), pinned(8*uintptr(n+1))
	defer outOff.free()
	defer status.free()
	defer hOff.free()
	if err := call("honu_encode_sizes", C.honu_encode_sizes(c.ctx, (*C.honu_meta)(d.rows.p),
		C.uint64_t(b.vars.n), (*C.honu_acl)(d.acls.p), C.uint64_t(b.nacl), (*C.uint32_t)(d.regs.p),
		C.uint64_t(b.nreg), (*C.uint64_t)(d.payOff.p), C.uint64_t(n), (*C.uint64_t)(outOff.p),
		(*C.int32_t)(status.p), c.stream)); err != nil {
		return nil, nil, err
	}
	// HONU_E_WORKSPACE here (n > the context's maxRecords) would leave outOff
	// unwritten: nothing below may read it then
	if err := call("honu_exclusive_scan", C.honu_exclusive_scan(c.ctx, (*C.uint64_t)(outOff.p),
		C.uint64_t(n), (*C.uint64_t)(outOff.p), c.stream)); err != nil {
		return nil, nil, err
	}
	if err := call("d2h", C.honu_memcpy_d2h(hOff.p, outOff.p, C.uint64_t(hOff.n), c.stream)); err != nil {
		return nil, nil, err
	}
	if err := call("sync", C.honu_stream_sync(c.stream)); err != nil {
		return nil, nil, err
	}
	offs := unsafe.Slice((*uint64)(hOff.p), n+1)
	// 4. encode into a device arena, copy the records back
	out := device(uintptr(offs[n]))
	defer out.free()
	if err := call("honu_encode", C.honu_encode(c.ctx, (*C.honu_meta)(d.rows.p),
		(*C.uint8_t)(d.vars.p), C.uint64_t(b.vars.n), (*C.honu_acl)(d.acls.p), C.uint64_t(b.nacl),
		(*C.uint32_t)(d.regs.p), C.uint64_t(b.nreg), (*C.uint8_t)(d.pay.p), (*C.uint64_t)(d.payOff.p),
		C.uint64_t(n), (*C.uint8_t)(out.p), C.uint64_t(out.n), (*C.uint64_t)(outOff.p),
		(*C.int32_t)(status.p), c.stream)); err != nil {
		return nil, nil, err
	}
	hOut, hSt := pinned(out.n), pinned(4*uintptr(n))
	defer hOut.free()
	defer hSt.free()
	for _, st := range []C.int32_t{
		C.honu_memcpy_d2h(hOut.p, out.p, C.uint64_t(out.n), c.stream),
		C.honu_memcpy_d2h(hSt.p, status.p, C.uint64_t(hSt.n), c.stream),
		C.honu_stream_sync(c.stream),
	} {
		if err := call("download", st); err != nil {
			return nil, nil, err
		}
	}
	objs, errs := make([]Object, n), make([]error, n)
	all, st := hOut.bytes(), unsafe.Slice((*int32)(hSt.p), n)
	for i := range objs {
		if errs[i] = recordErr(C.int32_t(st[i])); errs[i] != nil {
			continue
		}
		objs[i] = append(Object(nil), all[offs[i]:offs[i+1]]...) // caller-owned copy, like Marshal
	}
	return objs, errs, nil
}

// DecodeBatch is Object.Metadata + Object.Data for many records.
func (c *Codec) DecodeBatch(objs []Object) ([]*metadata.Metadata, [][]byte, []error, error) {
	n := len(objs)
	// 1. concatenate objs into a pinned arena with CSR offsets; upload
	var total uintptr
	for _, o := range objs {
		total += uintptr(len(o))
	}
	hArena, hOff := pinned(total), pinned(8*uintptr(n+1))
	defer hArena.free()
	defer hOff.free()
	arena, off := hArena.bytes(), unsafe.Slice((*uint64)(hOff.p), n+1)
	for i, o := range objs {
		off[i+1] = off[i] + uint64(copy(arena[off[i]:], o))
	}
	dArena, dOff := device(total), device(hOff.n)
	defer dArena.free()
	defer dOff.free()
	for _, st := range []C.int32_t{
		C.honu_memcpy_h2d(dArena.p, hArena.p, C.uint64_t(total), c.stream),
		C.honu_memcpy_h2d(dOff.p, hOff.p, C.uint64_t(hOff.n), c.stream),
	} {
		if err := call("upload", st); err != nil {
			return nil, nil, nil, err
		}
	}
	// 2. decode, zero copy: rows, record info, ACL / region tables. The tables
	//    are sized by ENTRY COUNTS, not record bytes (an entry takes >= 1 byte,
	//    so byte-sized tables would be 20 + 4 bytes per record byte: 24x the
	//    arena): start from the codec's running estimate, and when the batch
	//    needs more, the call's d_totals says exactly how many (records past a
	//    cap get HONU_ERR_CAPACITY and nothing else changes): re-allocate to the
	//    totals and decode again. An ACL list whose entries are all present
	//    comes back in place (HONU_ACL_INPLACE) and takes no table entry, and
	//    so does every region list (HONU_REGIONS_INPLACE): with the defaults
	//    only lists holding a nil ACL entry need the tables.
	//    honu_amd/c_abi_demo.c runs this flow in C.
	rows, info := device(uintptr(n)*uintptr(C.sizeof_honu_meta)), device(uintptr(n)*uintptr(C.sizeof_honu_record_info))
	tot, hTot := device(32), pinned(32)
	defer rows.free()
	defer info.free()
	defer tot.free()
	defer hTot.free()
	totals := unsafe.Slice((*uint64)(hTot.p), 4)
	aclCap, regCap := c.aclPerRecord*uint64(n)+64, c.regPerRecord*uint64(n)+64
	var acl, regs devBuf
	for try := 0; ; try++ {
		acl, regs = device(uintptr(aclCap)*uintptr(C.sizeof_honu_acl)), device(4*uintptr(regCap))
		if err := call("honu_decode_batch", C.honu_decode_batch(c.ctx, (*C.uint8_t)(dArena.p),
			(*C.uint64_t)(dOff.p), C.uint64_t(n), (*C.honu_meta)(rows.p), (*C.honu_record_info)(info.p),
			(*C.honu_acl)(acl.p), C.uint64_t(aclCap), (*C.uint32_t)(regs.p), C.uint64_t(regCap), nil, 0,
			(*C.uint64_t)(tot.p), c.stream)); err != nil {
			acl.free()
			regs.free()
			return nil, nil, nil, err // e.g. HONU_E_WORKSPACE: n > maxRecords, nothing was decoded
		}
		err := call("totals", C.honu_memcpy_d2h(hTot.p, tot.p, 24, c.stream))
		if err == nil {
			err = call("sync", C.honu_stream_sync(c.stream))
		}
		if err != nil {
			acl.free()
			regs.free()
			return nil, nil, nil, err
		}
		if totals[0] <= aclCap && totals[1] <= regCap {
			break
		}
		acl.free()
		regs.free()
		if try == 1 { // the totals of one batch do not change between calls
			return nil, nil, nil, fmt.Errorf("%w: ACL %d / regions %d", ErrCapacity, totals[0], totals[1])
		}
		aclCap, regCap = totals[0], totals[1]
	}
	defer acl.free()
	defer regs.free()
	c.aclPerRecord, c.regPerRecord = (totals[0]+uint64(n)-1)/uint64(n), (totals[1]+uint64(n)-1)/uint64(n)
	// 3. download rows, info, tables (the arena is already here: hArena)
	hRows, hInfo := pinned(rows.n), pinned(info.n)
	hAcl, hReg := pinned(uintptr(totals[0])*uintptr(C.sizeof_honu_acl)), pinned(4*uintptr(totals[1]))
	defer hRows.free()
	defer hInfo.free()
	defer hAcl.free()
	defer hReg.free()
	for _, st := range []C.int32_t{
		C.honu_memcpy_d2h(hRows.p, rows.p, C.uint64_t(rows.n), c.stream),
		C.honu_memcpy_d2h(hInfo.p, info.p, C.uint64_t(info.n), c.stream),
		C.honu_memcpy_d2h(hAcl.p, acl.p, C.uint64_t(hAcl.n), c.stream),
		C.honu_memcpy_d2h(hReg.p, regs.p, C.uint64_t(hReg.n), c.stream),
		C.honu_stream_sync(c.stream),
	} {
		if err := call("download", st); err != nil {
			return nil, nil, nil, err
		}
	}
	rs := unsafe.Slice((*C.honu_meta)(hRows.p), n)
	is := unsafe.Slice((*C.honu_record_info)(hInfo.p), n)
	as := unsafe.Slice((*C.honu_acl)(hAcl.p), totals[0])
	gs := unsafe.Slice((*uint32)(hReg.p), totals[1])
	metas, datas, errs := make([]*metadata.Metadata, n), make([][]byte, n), make([]error, n)
	for i := range objs {
		if errs[i] = recordErr(is[i].meta_status); errs[i] == nil { // else Metadata() returns nil, err
			metas[i] = unflatten(&rs[i], arena, as, gs)
		}
		if is[i].data_status == 0 && is[i].data_len > 0 { // Data(): a subslice of objs[i], as in Go
			b := uint64(is[i].data_off) - off[i]
			datas[i] = objs[i][b : b+uint64(is[i].data_len)]
		}
	}
	return metas, datas, errs, nil
}

// unflatten is the Go decoder's own construction from one decoded row: spans
// index the concatenated arena and are copied out (lani Decode copies frames,
// decode.go:50-51), a zero-length frame is nil (decode.go:37-39), ACL count 0
// is a nil slice (metadata.go:254), regions are always a non-nil slice
// (region.go:160), time 0 is time.Time{} (decode.go:224-237). An ACL list
// returned in place (HONU_ACL_INPLACE) is read from the arena: entry k is the
// 18 bytes 01 | ClientID | Permissions at acl_off + 18 k (acls.go:26-51);
// otherwise from the ACL table, where present == 0 is a nil entry. A region
// list returned in place (HONU_REGIONS_INPLACE) is read from the arena too.
func unflatten(r *C.honu_meta, arena []byte, acl []C.honu_acl, regs []uint32) *metadata.Metadata {
	frame := func(s C.honu_span) []byte {
		if s.len == 0 {
			return nil
		}
		return append([]byte(nil), arena[s.off:s.off+s.len]...)
	}
	ulidOf := func(b [16]C.uint8_t) (u ulid.ULID) {
		for k := range u {
			u[k] = byte(b[k])
		}
		return u
	}
	when := func(ns C.int64_t) time.Time {
		if ns == 0 {
			return time.Time{}
		}
		return time.Unix(0, int64(ns)).In(time.UTC)
	}
	p := uint32(r.present)
	if p&C.HONU_HAS_META == 0 {
		return &metadata.Metadata{} // nil-flag 0x00: a zero Metadata, no error (object.go:76-82)
	}
	m := &metadata.Metadata{
		ObjectID: ulidOf(r.object_id), CollectionID: ulidOf(r.collection_id),
		MIME: string(frame(r.mime)), Owner: ulidOf(r.owner), Group: ulidOf(r.group),
		Permissions: uint8(r.permissions), Flags: uint8(r.flags),
		Created: when(r.created), Modified: when(r.modified),
		WriteRegions: make(region.Regions, r.regions_count),
	}
	if p&C.HONU_HAS_VERSION != 0 {
		m.Version = &metadata.Version{
			Scalar:    lamport.Scalar{PID: uint32(r.pid), VID: uint64(r.vid)},
			Region:    region.Region(r.region),
			Tombstone: r.tombstone != 0,
			Created:   when(r.version_created),
		}
		if p&C.HONU_HAS_PARENT != 0 {
			m.Version.Parent = &lamport.Scalar{PID: uint32(r.parent_pid), VID: uint64(r.parent_vid)}
		}
	}
	if p&C.HONU_HAS_SCHEMA != 0 {
		m.Schema = &metadata.SchemaVersion{Name: string(frame(r.schema_name)),
			Major: uint32(r.schema_major), Minor: uint32(r.schema_minor), Patch: uint32(r.schema_patch)}
	}
	if r.acl_count > 0 {
		m.ACL = make([]*metadata.AccessControl, r.acl_count)
		if p&C.HONU_ACL_INPLACE != 0 {
			for k := range m.ACL {
				e := arena[uint64(r.acl_off)+18*uint64(k):][:18]
				var u ulid.ULID
				copy(u[:], e[1:17])
				m.ACL[k] = &metadata.AccessControl{ClientID: u, Permissions: e[17]}
			}
		} else {
			for k := range m.ACL {
				e := &acl[uint64(r.acl_off)+uint64(k)]
				if e.present != 0 { // a nil entry stays nil (acls.go:41-51)
					m.ACL[k] = &metadata.AccessControl{ClientID: ulidOf(e.client_id), Permissions: uint8(e.permissions)}
				}
			}
		}
	}
	if p&C.HONU_REGIONS_INPLACE != 0 {
		// in place: the list's uvarints in the arena, read as Regions.Decode
		// reads them (region.go:154-169 -> lani DecodeUint32: at most 5 bytes,
		// truncated to uint32, decode.go:127-146); the GPU decode validated them
		q := uint64(r.regions_off)
		for k := range m.WriteRegions {
			v, w := binary.Uvarint(arena[q:min(q+5, uint64(len(arena)))])
			m.WriteRegions[k] = region.Region(uint32(v))
			q += uint64(w)
		}
	} else {
		for k := range m.WriteRegions {
			m.WriteRegions[k] = region.Region(regs[uint64(r.regions_off)+uint64(k)])
		}
	}
	if p&C.HONU_HAS_PUBLISHER != 0 {
		m.Publisher = &metadata.Publisher{PublisherID: ulidOf(r.publisher_id), ClientID: ulidOf(r.client_id),
			IPAddress: net.IP(frame(r.ip_address)), UserAgent: string(frame(r.user_agent))}
	}
	if p&C.HONU_HAS_ENCRYPTION != 0 {
		m.Encryption = &metadata.Encryption{PublicKeyID: string(frame(r.public_key_id)),
			EncryptionKey: frame(r.encryption_key), HMACSecret: frame(r.hmac_secret), Signature: frame(r.signature),
			SealingAlgorithm:    metadata.EncryptionAlgorithm(r.sealing_alg),
			EncryptionAlgorithm: metadata.EncryptionAlgorithm(r.encryption_alg),
			SignatureAlgorithm:  metadata.EncryptionAlgorithm(r.signature_alg)}
	}
	if p&C.HONU_HAS_COMPRESSION != 0 {
		m.Compression = &metadata.Compression{Algorithm: metadata.CompressionAlgorithm(r.compression_alg),
			Level: int64(r.compression_level)}
	}
	return m
}
