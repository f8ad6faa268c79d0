// fecmodule.cpp -- zfec_amd._fec, the CPython surface of the engine.
//
// Mirrors /root/reference/zfec/_fecmodule.c: classes Encoder(k, m) and
// Decoder(k, m) with .k/.m, Encoder.encode(inblocks, desired_blocks_nums=None),
// Decoder.decode(blocks, blocknums), the exception Error and test_from_agl().
// Argument checking and error strings follow _fecmodule.c:82-97,148-198,
// 429-474; the inputs the reference mishandles (desired numbers >= m, decode
// numbers in [m, 255], duplicate numbers, non-contiguous buffers) raise Error
// here instead of reading out of bounds, hanging or aborting.
//
// The encode/decode work goes through libzfec_hip.so (fec_encode_ex /
// fec_decode_ex) with the GIL released, as the reference does around
// fec_encode/fec_decode (_fecmodule.c:221-223, 506-508).  Device-resident
// blocks (torch tensors) use encode_into/decode_into with raw device addresses;
// zfec_amd/__init__.py routes them there.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <malloc.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/zfec_hip.h"

static PyObject* py_fec_error;

namespace {

// Large outputs from host memory: each call's output `bytes` are fresh
// objects (_fecmodule.c:206-217, 496-503).  With glibc's default policy every
// block of more than a few MiB is served by fresh pages (mmap, or a heap top
// trimmed on free), so each call faults them in and each free unmaps them:
// a 64 MiB K=3/M=10 encode from bytes ran at 2.6 GB/s that way against
// 15.3 GB/s when freed blocks are reused.  Changing glibc's
// policy is process-wide, and the reference module never does it, so it is
// opt-in: with ZFEC_AMD_MALLOC=reuse in the environment the first call with
// blocks of at least 1 MiB sets M_MMAP_THRESHOLD 32 MiB (blocks under it come
// from the heap) and M_TRIM_THRESHOLD 1 GiB (that much free heap is kept), as
// zfec_amd.reuse_host_memory() does.  By default nothing is changed.
int g_mallopt_calls = 0;  // mallopt calls made by this module (_fec._mallopt_calls(), a test hook)

void reuse_freed_outputs(Py_ssize_t sz) {
    static std::once_flag once;
    if (sz < (Py_ssize_t(1) << 20)) return;
    std::call_once(once, [] {
        const char* e = getenv("ZFEC_AMD_MALLOC");
        if (!e || strcmp(e, "reuse") != 0) return;
        (void)mallopt(M_MMAP_THRESHOLD, 32 << 20);
        (void)mallopt(M_TRIM_THRESHOLD, 1 << 30);
        g_mallopt_calls += 2;
    });
}

struct Coder {
    PyObject_HEAD
    unsigned short kk;
    unsigned short mm;
    fec_t* fec_matrix;
};

PyObject* Coder_new(PyTypeObject* type, PyObject*, PyObject*) {
    Coder* self = reinterpret_cast<Coder*>(type->tp_alloc(type, 0));
    if (self) {
        self->kk = 0;
        self->mm = 0;
        self->fec_matrix = nullptr;
    }
    return reinterpret_cast<PyObject*>(self);
}

int coder_init(Coder* self, PyObject* args, PyObject* kwdict, const char* fmt) {
    static const char* kwlist[] = {"k", "m", nullptr};
    int ink, inm;
    if (!PyArg_ParseTupleAndKeywords(args, kwdict, fmt, const_cast<char**>(kwlist), &ink, &inm)) return -1;
    // zfec/_fecmodule.c:82-97
    if (ink < 1) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: first argument is required to be greater than or equal to 1, but it was %d",
                     ink);
        return -1;
    }
    if (inm < 1) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: second argument is required to be greater than or equal to 1, but it was %d",
                     inm);
        return -1;
    }
    if (inm > 256) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: second argument is required to be less than or equal to 256, but it was %d",
                     inm);
        return -1;
    }
    if (ink > inm) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: first argument is required to be less than or equal to the second "
                     "argument, but they were %d and %d respectively",
                     ink, inm);
        return -1;
    }
    if (self->fec_matrix) {
        fec_free(self->fec_matrix);
        self->fec_matrix = nullptr;
    }
    self->kk = static_cast<unsigned short>(ink);
    self->mm = static_cast<unsigned short>(inm);
    fec_t* f;
    Py_BEGIN_ALLOW_THREADS f = fec_new(self->kk, self->mm);
    Py_END_ALLOW_THREADS if (!f) {
        PyErr_Format(py_fec_error, "fec_new failed: %s", fec_last_error_message());
        return -1;
    }
    self->fec_matrix = f;
    return 0;
}

int Encoder_init(Coder* self, PyObject* args, PyObject* kw) { return coder_init(self, args, kw, "ii:Encoder.__init__"); }
int Decoder_init(Coder* self, PyObject* args, PyObject* kw) { return coder_init(self, args, kw, "ii:Decoder.__init__"); }

void Coder_dealloc(Coder* self) {
    if (self->fec_matrix) fec_free(self->fec_matrix);
    Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

bool ready(Coder* self) {
    if (!self->fec_matrix) {
        PyErr_SetString(py_fec_error, "coder is not initialised");
        return false;
    }
    return true;
}

// Holds acquired buffers (at most 256: k <= 256) and releases them on scope
// exit.  Fixed arrays on the stack here and below: a small call's host cost
// is counted in microseconds, and growing vectors cost a dozen allocations.
struct Buffers {
    Py_buffer v[256];
    size_t n;
    explicit Buffers(size_t cnt) : n(cnt) {
        for (size_t i = 0; i < n; ++i) v[i].obj = nullptr;
    }
    ~Buffers() {
        for (size_t i = 0; i < n; ++i)
            if (v[i].obj) PyBuffer_Release(&v[i]);
    }
};

// Parse a sequence of ints into `out`; false with an exception set.
bool parse_nums(PyObject* fast, std::vector<long>& out) {
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    PyObject** items = PySequence_Fast_ITEMS(fast);
    out.resize(static_cast<size_t>(n));
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (!PyLong_Check(items[i])) {
            PyErr_Format(py_fec_error, "Precondition violation: second argument is required to contain int.");
            return false;
        }
        out[i] = PyLong_AsLong(items[i]);
        if (out[i] == -1 && PyErr_Occurred()) return false;
    }
    return true;
}

int raise_status(int st) {
    PyErr_Format(py_fec_error, "zfec-hip error %d: %s", st, fec_last_error_message());
    return -1;
}

// zfec_amd.Encoder / Decoder (the Python subclasses) take device tensors too:
// a first block with no buffer protocol whose .is_cuda is true routes the
// call to the subclass's _encode_device / _decode_device.  Checked here
// rather than in a Python override of encode/decode, so a call on bytes
// enters C directly (one Python frame less per small call).  Returns 1 with
// the result in *out, 0 if not routed, -1 with an exception set.
int route_device(PyObject* self, PyObject* blocks, const char* method, PyObject* a2, PyObject** out) {
    if (!PyObject_HasAttrString(self, method)) return 0;  // the bare _fec type
    PyObject* first = PySequence_Check(blocks) ? PySequence_GetItem(blocks, 0) : nullptr;
    if (!first) {
        PyErr_Clear();
        return 0;
    }
    int routed = 0;
    if (!PyObject_CheckBuffer(first)) {
        PyObject* cuda = PyObject_GetAttrString(first, "is_cuda");
        if (!cuda) {
            PyErr_Clear();
        } else {
            routed = PyObject_IsTrue(cuda) == 1;
            Py_DECREF(cuda);
        }
    }
    Py_DECREF(first);
    if (!routed) return 0;
    *out = PyObject_CallMethod(self, method, "OO", blocks, a2 ? a2 : Py_None);
    return *out ? 1 : -1;
}

// ---- Encoder.encode -----------------------------------------------------------
// zfec/_fecmodule.c:116-260
PyObject* Encoder_encode(Coder* self, PyObject* args) {
    PyObject* inblocks;
    PyObject* desired = nullptr;
    if (!PyArg_ParseTuple(args, "O|O:Encoder.encode", &inblocks, &desired)) return nullptr;
    if (!ready(self)) return nullptr;
    {
        PyObject* routed = nullptr;
        const int rd = route_device(reinterpret_cast<PyObject*>(self), inblocks, "_encode_device", desired, &routed);
        if (rd) return rd > 0 ? routed : nullptr;
    }
    const unsigned k = self->kk, m = self->mm;

    thread_local std::vector<long> nums;  // reused: no allocation per call
    nums.clear();
    if (desired && desired != Py_None) {
        PyObject* fd = PySequence_Fast(desired, "Second argument (optional) was not a sequence.");
        if (!fd) return nullptr;
        const bool ok = parse_nums(fd, nums);
        Py_DECREF(fd);
        if (!ok) return nullptr;
        for (long x : nums)
            if (x < 0 || x >= static_cast<long>(m)) {
                PyErr_Format(py_fec_error,
                             "Precondition violation: desired block nums are required to be in [0, m-1] = [0, %u], "
                             "but one was %ld",
                             m - 1, x);
                return nullptr;
            }
    } else {
        nums.resize(m);
        for (unsigned i = 0; i < m; ++i) nums[i] = i;
    }

    PyObject* fast = PySequence_Fast(inblocks, "First argument was not a sequence.");
    if (!fast) return nullptr;
    if (PySequence_Fast_GET_SIZE(fast) != static_cast<Py_ssize_t>(k)) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: Wrong length -- first argument (the sequence of input blocks) is required "
                     "to contain exactly k blocks.  len(first): %zd, k: %d",
                     PySequence_Fast_GET_SIZE(fast), int(k));
        Py_DECREF(fast);
        return nullptr;
    }
    PyObject** items = PySequence_Fast_ITEMS(fast);
    Buffers bufs(k);
    const gf* in[256];
    Py_ssize_t sz = -1;
    for (unsigned i = 0; i < k; ++i) {
        if (PyObject_GetBuffer(items[i], &bufs.v[i], PyBUF_SIMPLE)) {
            bufs.v[i].obj = nullptr;
            Py_DECREF(fast);
            return nullptr;
        }
        if (!PyBuffer_IsContiguous(&bufs.v[i], 'C')) {
            PyErr_Format(py_fec_error, "Precondition violation: Input blocks are required to be C-contiguous.");
            Py_DECREF(fast);
            return nullptr;
        }
        if (sz >= 0 && sz != bufs.v[i].len) {
            PyErr_Format(py_fec_error,
                         "Precondition violation: Input blocks are required to be all the same length.  length of one "
                         "block was: %zd, length of another block was: %zd",
                         sz, bufs.v[i].len);
            Py_DECREF(fast);
            return nullptr;
        }
        sz = bufs.v[i].len;
        in[i] = static_cast<const gf*>(bufs.v[i].buf);
    }
    if (sz < 0) sz = 0;

    // one fresh bytes object per requested secondary block (_fecmodule.c:206-217)
    reuse_freed_outputs(sz);
    // desired numbers may repeat (the reference allows it): up to nums.size() outputs
    std::vector<unsigned> ids_big;
    std::vector<PyObject*> produced_big;
    std::vector<gf*> outp_big;
    unsigned ids_s[256];
    PyObject* produced_s[256];
    gf* outp_s[256];
    unsigned* ids = ids_s;
    PyObject** produced = produced_s;
    gf** outp = outp_s;
    if (nums.size() > 256) {
        ids_big.resize(nums.size());
        produced_big.resize(nums.size());
        outp_big.resize(nums.size());
        ids = ids_big.data();
        produced = produced_big.data();
        outp = outp_big.data();
    }
    size_t nout = 0;
    for (long x : nums)
        if (x >= static_cast<long>(k)) {
            PyObject* b = PyBytes_FromStringAndSize(nullptr, sz);
            if (!b) {
                for (size_t i = 0; i < nout; ++i) Py_DECREF(produced[i]);
                Py_DECREF(fast);
                return nullptr;
            }
            ids[nout] = static_cast<unsigned>(x);
            produced[nout] = b;
            outp[nout] = reinterpret_cast<gf*>(PyBytes_AS_STRING(b));
            ++nout;
        }
    int st = FEC_OK;
    if (nout) {
        Py_BEGIN_ALLOW_THREADS st = fec_encode_ex(self->fec_matrix, in, outp, ids, nout, static_cast<size_t>(sz), nullptr,
                                                  FEC_FLAG_LIBRARY_STREAM | FEC_FLAG_HOST_MEMORY);
        Py_END_ALLOW_THREADS
    }
    if (st != FEC_OK) {
        for (size_t i = 0; i < nout; ++i) Py_DECREF(produced[i]);
        Py_DECREF(fast);
        raise_status(st);
        return nullptr;
    }
    PyObject* result = PyList_New(static_cast<Py_ssize_t>(nums.size()));
    if (!result) {
        for (size_t i = 0; i < nout; ++i) Py_DECREF(produced[i]);
        Py_DECREF(fast);
        return nullptr;
    }
    size_t ci = 0;
    for (size_t i = 0; i < nums.size(); ++i) {
        if (nums[i] < static_cast<long>(k)) {  // primaries by reference (_fecmodule.c:231-235)
            PyObject* o = items[nums[i]];
            Py_INCREF(o);
            PyList_SET_ITEM(result, static_cast<Py_ssize_t>(i), o);
        } else {
            PyList_SET_ITEM(result, static_cast<Py_ssize_t>(i), produced[ci++]);
        }
    }
    Py_DECREF(fast);
    return result;
}

// ---- Decoder.decode -----------------------------------------------------------
// zfec/_fecmodule.c:400-544
PyObject* Decoder_decode(Coder* self, PyObject* args) {
    PyObject *blocks, *blocknums;
    if (!PyArg_ParseTuple(args, "OO:Decoder.decode", &blocks, &blocknums)) return nullptr;
    if (!ready(self)) return nullptr;
    {
        PyObject* routed = nullptr;
        const int rd = route_device(reinterpret_cast<PyObject*>(self), blocks, "_decode_device", blocknums, &routed);
        if (rd) return rd > 0 ? routed : nullptr;
    }
    const unsigned k = self->kk, m = self->mm;

    PyObject* fb = PySequence_Fast(blocks, "First argument was not a sequence.");
    if (!fb) return nullptr;
    PyObject* fn = PySequence_Fast(blocknums, "Second argument was not a sequence.");
    if (!fn) {
        Py_DECREF(fb);
        return nullptr;
    }
    struct Drop {
        PyObject *a, *b;
        ~Drop() {
            Py_XDECREF(a);
            Py_XDECREF(b);
        }
    } drop{fb, fn};

    if (PySequence_Fast_GET_SIZE(fb) != static_cast<Py_ssize_t>(k)) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: Wrong length -- first argument is required to contain exactly k blocks.  "
                     "len(first): %zd, k: %d",
                     PySequence_Fast_GET_SIZE(fb), int(k));
        return nullptr;
    }
    if (PySequence_Fast_GET_SIZE(fn) != static_cast<Py_ssize_t>(k)) {
        PyErr_Format(py_fec_error,
                     "Precondition violation: Wrong length -- blocknums is required to contain exactly k blocks.  "
                     "len(blocknums): %zd, k: %d",
                     PySequence_Fast_GET_SIZE(fn), int(k));
        return nullptr;
    }
    thread_local std::vector<long> nums;  // reused: no allocation per call
    if (!parse_nums(fn, nums)) return nullptr;
    unsigned char seen[256] = {};
    for (long x : nums) {
        if (x < 0 || x > 255) {  // _fecmodule.c:459-462
            PyErr_Format(py_fec_error,
                         "Precondition violation: block nums can't be less than zero or greater than 255.  %ld\n", x);
            return nullptr;
        }
        if (x >= static_cast<long>(m)) {
            PyErr_Format(py_fec_error,
                         "Precondition violation: block nums are required to be less than m = %u, but one was %ld", m, x);
            return nullptr;
        }
        if (seen[x]) {
            PyErr_Format(py_fec_error, "Precondition violation: block nums are required to be distinct, but %ld repeats",
                         x);
            return nullptr;
        }
        seen[x] = 1;
    }
    PyObject** items = PySequence_Fast_ITEMS(fb);
    Buffers bufs(k);
    const gf* cblocks[256];
    PyObject* objs[256];
    unsigned cnums[256];
    std::copy(items, items + k, objs);
    Py_ssize_t sz = -1;
    for (unsigned i = 0; i < k; ++i) {
        if (PyObject_GetBuffer(items[i], &bufs.v[i], PyBUF_SIMPLE)) {
            bufs.v[i].obj = nullptr;
            return nullptr;
        }
        if (!PyBuffer_IsContiguous(&bufs.v[i], 'C')) {
            PyErr_Format(py_fec_error, "Precondition violation: Input blocks are required to be C-contiguous.");
            return nullptr;
        }
        if (sz >= 0 && sz != bufs.v[i].len) {
            PyErr_Format(py_fec_error,
                         "Precondition violation: Input blocks are required to be all the same length.  length of one "
                         "block was: %zd, length of another block was: %zd\n",
                         sz, bufs.v[i].len);
            return nullptr;
        }
        sz = bufs.v[i].len;
        cblocks[i] = static_cast<const gf*>(bufs.v[i].buf);
        cnums[i] = static_cast<unsigned>(nums[i]);
    }
    if (sz < 0) sz = 0;
    // move primary i to slot i (_fecmodule.c:482-493); numbers are distinct, so this terminates
    for (unsigned i = 0; i < k;) {
        if (cnums[i] >= k || cnums[i] == i) {
            ++i;
        } else {
            const unsigned c = cnums[i];
            std::swap(cnums[i], cnums[c]);
            std::swap(cblocks[i], cblocks[c]);
            std::swap(objs[i], objs[c]);
        }
    }
    PyObject* rec[256];
    gf* recp[256];
    size_t nrec = 0;
    reuse_freed_outputs(sz);
    for (unsigned i = 0; i < k; ++i)
        if (cnums[i] >= k) {
            PyObject* b = PyBytes_FromStringAndSize(nullptr, sz);
            if (!b) {
                for (size_t q = 0; q < nrec; ++q) Py_DECREF(rec[q]);
                return nullptr;
            }
            rec[nrec] = b;
            recp[nrec++] = reinterpret_cast<gf*>(PyBytes_AS_STRING(b));
        }
    int st = FEC_OK;
    if (nrec) {
        Py_BEGIN_ALLOW_THREADS st = fec_decode_ex(self->fec_matrix, cblocks, recp, cnums, static_cast<size_t>(sz), nullptr,
                                                  FEC_FLAG_LIBRARY_STREAM | FEC_FLAG_HOST_MEMORY);
        Py_END_ALLOW_THREADS
    }
    if (st != FEC_OK) {
        for (size_t q = 0; q < nrec; ++q) Py_DECREF(rec[q]);
        raise_status(st);
        return nullptr;
    }
    PyObject* result = PyList_New(k);
    if (!result) {
        for (size_t q = 0; q < nrec; ++q) Py_DECREF(rec[q]);
        return nullptr;
    }
    size_t ri = 0;
    for (unsigned i = 0; i < k; ++i) {
        if (cnums[i] == i) {
            Py_INCREF(objs[i]);
            PyList_SET_ITEM(result, i, objs[i]);
        } else {
            PyList_SET_ITEM(result, i, rec[ri++]);
        }
    }
    return result;
}

// ---- device-address entry points (used by zfec_amd for torch tensors) ---------

bool addr_list(PyObject* seq, std::vector<void*>& out, const char* what) {
    PyObject* f = PySequence_Fast(seq, what);
    if (!f) return false;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(f);
    out.resize(static_cast<size_t>(n));
    for (Py_ssize_t i = 0; i < n; ++i) {
        out[i] = PyLong_AsVoidPtr(PySequence_Fast_GET_ITEM(f, i));
        if (PyErr_Occurred()) {
            Py_DECREF(f);
            return false;
        }
    }
    Py_DECREF(f);
    return true;
}

bool uint_list(PyObject* seq, std::vector<unsigned>& out, const char* what) {
    PyObject* f = PySequence_Fast(seq, what);
    if (!f) return false;
    std::vector<long> v;
    const bool ok = parse_nums(f, v);
    Py_DECREF(f);
    if (!ok) return false;
    out.assign(v.begin(), v.end());
    for (long x : v)
        if (x < 0 || x > 255) {
            PyErr_Format(py_fec_error, "Precondition violation: block nums can't be less than zero or greater than 255.  %ld\n", x);
            return false;
        }
    return true;
}

// encode_into(in_addrs, out_addrs, block_nums, sz, stream=0, sync=False)
PyObject* Encoder_encode_into(Coder* self, PyObject* args, PyObject* kw) {
    static const char* kwlist[] = {"in_addrs", "out_addrs", "block_nums", "sz", "stream", "sync", nullptr};
    PyObject *pin, *pout, *pnums;
    unsigned long long sz = 0, stream = 0;
    int sync = 0;
    if (!PyArg_ParseTupleAndKeywords(args, kw, "OOOK|Kp:Encoder.encode_into", const_cast<char**>(kwlist), &pin, &pout,
                                     &pnums, &sz, &stream, &sync))
        return nullptr;
    if (!ready(self)) return nullptr;
    std::vector<void*> in, out;
    std::vector<unsigned> nums;
    if (!addr_list(pin, in, "in_addrs must be a sequence") || !addr_list(pout, out, "out_addrs must be a sequence") ||
        !uint_list(pnums, nums, "block_nums must be a sequence"))
        return nullptr;
    if (in.size() != self->kk || out.size() != nums.size()) {
        PyErr_Format(py_fec_error, "Precondition violation: need k=%d inputs and one output per block num", int(self->kk));
        return nullptr;
    }
    int st;
    Py_BEGIN_ALLOW_THREADS st = fec_encode_ex(self->fec_matrix, reinterpret_cast<const gf* const*>(in.data()),
                                              reinterpret_cast<gf* const*>(out.data()), nums.data(), nums.size(), sz,
                                              reinterpret_cast<void*>(stream), sync ? 0u : FEC_FLAG_ASYNC);
    Py_END_ALLOW_THREADS if (st != FEC_OK) {
        raise_status(st);
        return nullptr;
    }
    Py_RETURN_NONE;
}

// decode_into(in_addrs, out_addrs, slot_nums, sz, stream=0, sync=False): slots already ordered
PyObject* Decoder_decode_into(Coder* self, PyObject* args, PyObject* kw) {
    static const char* kwlist[] = {"in_addrs", "out_addrs", "slot_nums", "sz", "stream", "sync", nullptr};
    PyObject *pin, *pout, *pnums;
    unsigned long long sz = 0, stream = 0;
    int sync = 0;
    if (!PyArg_ParseTupleAndKeywords(args, kw, "OOOK|Kp:Decoder.decode_into", const_cast<char**>(kwlist), &pin, &pout,
                                     &pnums, &sz, &stream, &sync))
        return nullptr;
    if (!ready(self)) return nullptr;
    std::vector<void*> in, out;
    std::vector<unsigned> nums;
    if (!addr_list(pin, in, "in_addrs must be a sequence") || !addr_list(pout, out, "out_addrs must be a sequence") ||
        !uint_list(pnums, nums, "slot_nums must be a sequence"))
        return nullptr;
    if (in.size() != self->kk || nums.size() != self->kk) {
        PyErr_Format(py_fec_error, "Precondition violation: need k=%d inputs and slot nums", int(self->kk));
        return nullptr;
    }
    int st;
    Py_BEGIN_ALLOW_THREADS st = fec_decode_ex(self->fec_matrix, reinterpret_cast<const gf* const*>(in.data()),
                                              reinterpret_cast<gf* const*>(out.data()), nums.data(), sz,
                                              reinterpret_cast<void*>(stream), sync ? 0u : FEC_FLAG_ASYNC);
    Py_END_ALLOW_THREADS if (st != FEC_OK) {
        raise_status(st);
        return nullptr;
    }
    Py_RETURN_NONE;
}

PyObject* Coder_enc_matrix(Coder* self, PyObject*) {
    if (!ready(self)) return nullptr;
    return PyBytes_FromStringAndSize(reinterpret_cast<const char*>(self->fec_matrix->enc_matrix),
                                     Py_ssize_t(self->kk) * self->mm);
}

const char Encoder_doc[] =
    "Encoder(k, m): systematic Reed-Solomon encoder over GF(2^8) running on MI355X.\n\n"
    "@param k: the number of packets required for reconstruction\n"
    "@param m: the number of packets generated\n";
const char Decoder_doc[] =
    "Decoder(k, m): recovers the k primary blocks from any k of the m blocks (MI355X).\n\n"
    "@param k: the number of packets required for reconstruction\n"
    "@param m: the number of packets generated\n";
const char encode_doc[] =
    "encode(inblocks, desired_blocks_nums=None) -> list of blocks.\n"
    "Primary blocks in the result are the very objects passed in; secondary blocks are new bytes.";
const char decode_doc[] =
    "decode(blocks, blocknums) -> the k primary blocks in order.\n"
    "Primary blocks present in the input are returned by reference; recovered ones are new bytes.";

PyMethodDef Encoder_methods[] = {
    {"encode", reinterpret_cast<PyCFunction>(Encoder_encode), METH_VARARGS, encode_doc},
    {"encode_into", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(Encoder_encode_into)),
     METH_VARARGS | METH_KEYWORDS, "Encode device-resident blocks given raw device addresses (stream-ordered)."},
    {"enc_matrix", reinterpret_cast<PyCFunction>(Coder_enc_matrix), METH_NOARGS, "The m x k encoding matrix as bytes."},
    {nullptr, nullptr, 0, nullptr}};
PyMethodDef Decoder_methods[] = {
    {"decode", reinterpret_cast<PyCFunction>(Decoder_decode), METH_VARARGS, decode_doc},
    {"decode_into", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(Decoder_decode_into)),
     METH_VARARGS | METH_KEYWORDS, "Decode device-resident blocks given raw device addresses (stream-ordered)."},
    {"enc_matrix", reinterpret_cast<PyCFunction>(Coder_enc_matrix), METH_NOARGS, "The m x k encoding matrix as bytes."},
    {nullptr, nullptr, 0, nullptr}};
PyMemberDef Coder_members[] = {
    {const_cast<char*>("k"), T_USHORT, offsetof(Coder, kk), READONLY, const_cast<char*>("k")},
    {const_cast<char*>("m"), T_USHORT, offsetof(Coder, mm), READONLY, const_cast<char*>("m")},
    {nullptr, 0, 0, 0, nullptr}};

PyTypeObject Encoder_type = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject Decoder_type = {PyVarObject_HEAD_INIT(nullptr, 0)};

// zfec/_fecmodule.c:614-659: k=3, n=5, 8-byte blocks of 0x01/0x02/0x03; encode
// blocks 3 and 4, decode primaries 0 and 1 from {3, 4, 2}, compare.
PyObject* test_from_agl(PyObject*, PyObject*) {
    unsigned char b0[8], b1[8], b2[8], b3[8], b4[8], b0c[8], b1c[8];
    std::memset(b0, 1, 8);
    std::memset(b1, 2, 8);
    std::memset(b2, 3, 8);
    const gf* blocks[3] = {b0, b1, b2};
    gf* outblocks[2] = {b3, b4};
    unsigned block_nums[2] = {3, 4};
    fec_t* f = fec_new(3, 5);
    if (!f) return PyErr_Format(py_fec_error, "fec_new: %s", fec_last_error_message());
    int st = fec_encode_ex(f, blocks, outblocks, block_nums, 2, 8, nullptr, FEC_FLAG_LIBRARY_STREAM);
    std::memcpy(b0c, b0, 8);
    std::memcpy(b1c, b1, 8);
    const gf* inpkts[3] = {b3, b4, b2};
    gf* outpkts[2] = {b0, b1};
    unsigned indexes[3] = {3, 4, 2};
    if (st == FEC_OK) st = fec_decode_ex(f, inpkts, outpkts, indexes, 8, nullptr, FEC_FLAG_LIBRARY_STREAM);
    if (st != FEC_OK) {
        raise_status(st);  // before fec_free, which resets the thread's status
        fec_free(f);
        return nullptr;
    }
    fec_free(f);
    if (std::memcmp(b0, b0c, 8) == 0 && std::memcmp(b1, b1c, 8) == 0) Py_RETURN_TRUE;
    Py_RETURN_FALSE;
}

// batch_call(kind, code, src, sbs, sss, dst, dbs, dss, nums, sz, nstripes, stream, flags) -> status
//
// fec_encode_batch (kind 0) / fec_decode_batch (kind 1) of the C-ABI, called
// from C: `code` is a fec_t* from fec_new, buffers and the stream are raw
// addresses, `nums` a tuple or list of block numbers (decode: the k slot
// numbers).  Returns the call's status (fec_last_error_message holds the
// message).  zfec_amd.capi routes its batched calls here: ctypes' conversion
// of the thirteen arguments cost ~2 us of the ~5 us host enqueue of a batched
// launch (BENCH_r02 host_enqueue_us 5.1 vs 3.2 from C, tools/host_cost.hip).
PyObject* py_batch_call(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
    if (nargs != 13) {
        PyErr_Format(PyExc_TypeError, "batch_call takes 13 arguments (%zd given)", nargs);
        return nullptr;
    }
    size_t v[13] = {};
    for (int i = 0; i < 13; ++i) {
        if (i == 8) continue;
        v[i] = PyLong_AsSize_t(args[i]);
        if (v[i] == size_t(-1) && PyErr_Occurred()) return nullptr;
    }
    if (v[0] > 1) {
        PyErr_Format(PyExc_ValueError, "batch_call: kind must be 0 (encode) or 1 (decode), not %zu", v[0]);
        return nullptr;
    }
    PyObject* seq = PySequence_Fast(args[8], "batch_call: nums must be a tuple or list");
    if (!seq) return nullptr;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    unsigned nums[256];
    if (n > 256) {
        Py_DECREF(seq);
        PyErr_SetString(py_fec_error, "Precondition violation: at most 256 block numbers");
        return nullptr;
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
        const unsigned long x = PyLong_AsUnsignedLong(PySequence_Fast_GET_ITEM(seq, i));
        if (x == static_cast<unsigned long>(-1) && PyErr_Occurred()) {
            Py_DECREF(seq);
            return nullptr;
        }
        nums[i] = x > 0xffffffffu ? 0xffffffffu : static_cast<unsigned>(x);  // out of range: the library rejects it
    }
    Py_DECREF(seq);
    // decode reads k slot numbers: missing ones are out of range (rejected)
    for (Py_ssize_t i = n; i < 256; ++i) nums[i] = 0xffffffffu;
    const fec_t* code = reinterpret_cast<const fec_t*>(v[1]);
    const gf* src = reinterpret_cast<const gf*>(v[2]);
    gf* dst = reinterpret_cast<gf*>(v[5]);
    void* stream = reinterpret_cast<void*>(v[11]);
    const unsigned flags = static_cast<unsigned>(v[12]);
    int st;
    if (v[0] == 0) {
        Py_BEGIN_ALLOW_THREADS st = fec_encode_batch(code, src, v[3], v[4], dst, v[6], v[7], nums, size_t(n), v[9],
                                                     v[10], stream, flags);
        Py_END_ALLOW_THREADS
    } else {
        Py_BEGIN_ALLOW_THREADS st = fec_decode_batch(code, src, v[3], v[4], dst, v[6], v[7], nums, v[9], v[10],
                                                     stream, flags);
        Py_END_ALLOW_THREADS
    }
    return PyLong_FromLong(st);
}

PyObject* py_device_count(PyObject*, PyObject*) { return PyLong_FromLong(fec_device_count()); }
PyObject* py_version(PyObject*, PyObject*) { return PyUnicode_FromString(fec_version()); }
PyObject* py_mallopt_calls(PyObject*, PyObject*) { return PyLong_FromLong(g_mallopt_calls); }

PyMethodDef module_functions[] = {
    {"_mallopt_calls", py_mallopt_calls, METH_NOARGS,
     "mallopt calls this module has made (0 unless ZFEC_AMD_MALLOC=reuse; a test hook)."},
    {"test_from_agl", test_from_agl, METH_NOARGS, "Encode/decode round trip of zfec's C self-test (on the GPU)."},
    {"device_count", py_device_count, METH_NOARGS, "Number of visible GPUs."},
    {"version", py_version, METH_NOARGS, "Library version."},
    {"batch_call", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_batch_call)), METH_FASTCALL,
     "batch_call(kind, code, src, sbs, sss, dst, dbs, dss, nums, sz, nstripes, stream, flags) -> status: "
     "fec_encode_batch (kind 0) / fec_decode_batch (kind 1) with raw addresses."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moduledef = {PyModuleDef_HEAD_INIT, "_fec", "FEC - Forward Error Correction on MI355X", -1,
                         module_functions};

void fill_type(PyTypeObject& t, const char* name, const char* doc, initproc init, PyMethodDef* methods) {
    t.tp_name = name;
    t.tp_basicsize = sizeof(Coder);
    t.tp_dealloc = reinterpret_cast<destructor>(Coder_dealloc);
    t.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE;
    t.tp_doc = doc;
    t.tp_methods = methods;
    t.tp_members = Coder_members;
    t.tp_init = init;
    t.tp_new = Coder_new;
}

}  // namespace

PyMODINIT_FUNC PyInit__fec(void) {
    fill_type(Encoder_type, "zfec_amd._fec.Encoder", Encoder_doc, reinterpret_cast<initproc>(Encoder_init),
              Encoder_methods);
    fill_type(Decoder_type, "zfec_amd._fec.Decoder", Decoder_doc, reinterpret_cast<initproc>(Decoder_init),
              Decoder_methods);
    if (PyType_Ready(&Encoder_type) < 0 || PyType_Ready(&Decoder_type) < 0) return nullptr;
    PyObject* module = PyModule_Create(&moduledef);
    if (!module) return nullptr;
    Py_INCREF(&Encoder_type);
    Py_INCREF(&Decoder_type);
    PyModule_AddObject(module, "Encoder", reinterpret_cast<PyObject*>(&Encoder_type));
    PyModule_AddObject(module, "Decoder", reinterpret_cast<PyObject*>(&Decoder_type));
    py_fec_error = PyErr_NewException("zfec_amd.Error", nullptr, nullptr);
    Py_INCREF(py_fec_error);
    PyModule_AddObject(module, "Error", py_fec_error);
    fec_init();
    return module;
}
