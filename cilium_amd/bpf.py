"""Python mirror of Cilium's ``pkg/bpf`` on top of libgpuflow.

Same names, argument meaning and error behaviour as the Go package
(/root/reference/pkg/bpf/bpf.go, map.go): the raw calls return/raise the way
``bpf.UpdateElement`` & co. do, with the kernel errno inside the message.
"""
import ctypes as C
import errno
import os

import numpy as np

from ._lib import lib, gf_map_info

# pkg/bpf/bpf.go:38-52
BPF_MAP_TYPE_UNSPEC = 0
BPF_MAP_TYPE_HASH = 1
BPF_MAP_TYPE_ARRAY = 2
BPF_MAP_TYPE_PROG_ARRAY = 3
BPF_MAP_TYPE_PERF_EVENT_ARRAY = 4
BPF_MAP_TYPE_PERCPU_HASH = 5
BPF_MAP_TYPE_PERCPU_ARRAY = 6
BPF_MAP_TYPE_STACK_TRACE = 7
BPF_MAP_TYPE_CGROUP_ARRAY = 8
BPF_MAP_TYPE_LRU_HASH = 9
BPF_MAP_TYPE_LRU_PERCPU_HASH = 10
BPF_MAP_TYPE_LPM_TRIE = 11
# pkg/bpf/bpf.go:73-78
BPF_ANY = 0
BPF_NOEXIST = 1
BPF_EXIST = 2
BPF_F_NO_PREALLOC = 1 << 0
BPF_F_NO_COMMON_LRU = 1 << 1

MapTypeHash = BPF_MAP_TYPE_HASH
MapTypeLRUHash = BPF_MAP_TYPE_LRU_HASH
MapTypeLPMTrie = BPF_MAP_TYPE_LPM_TRIE

# pkg/bpf/bpffs.go:35-38
MAP_PREFIX = "/sys/fs/bpf/tc/globals"


def MapPath(name):
    return os.path.join(MAP_PREFIX, name)


class BPFError(OSError):
    pass


def _err(msg, rc):
    e = -rc
    return BPFError(e, f"{msg}: {os.strerror(e)}")


def _buf(b, size=None):
    if isinstance(b, (bytes, bytearray)):
        if size is not None and len(b) != size:
            raise ValueError(f"buffer of {len(b)} bytes, expected {size}")
        return C.create_string_buffer(bytes(b), len(b))
    return b


def CreateMap(mapType, keySize, valueSize, maxEntries, flags=0):
    """bpf.CreateMap, pkg/bpf/bpf.go:84-112: returns the handle (> 0)."""
    rc = lib.gf_map_create(mapType, keySize, valueSize, maxEntries, flags)
    if rc <= 0:
        raise _err("Unable to create map", rc if rc < 0 else -errno.EINVAL)
    return rc


def UpdateElement(fd, key, value, flags=BPF_ANY):
    """bpf.UpdateElement, pkg/bpf/bpf.go:129-149."""
    rc = lib.gf_map_update_elem(fd, _buf(key), _buf(value), flags)
    if rc:
        raise _err("Unable to update element", rc)


def LookupElement(fd, key, valueSize):
    """bpf.LookupElement, pkg/bpf/bpf.go:153-172: returns the value bytes."""
    v = C.create_string_buffer(valueSize)
    rc = lib.gf_map_lookup_elem(fd, _buf(key), v)
    if rc:
        raise _err("Unable to lookup element", rc)
    return v.raw


def DeleteElement(fd, key):
    """bpf.DeleteElement, pkg/bpf/bpf.go:175-192."""
    rc = lib.gf_map_delete_elem(fd, _buf(key))
    if rc:
        raise _err("Unable to delete element", rc)


def GetNextKey(fd, key, keySize):
    """bpf.GetNextKey, pkg/bpf/bpf.go:195-213 (key None -> first key)."""
    nk = C.create_string_buffer(keySize)
    rc = lib.gf_map_get_next_key(fd, _buf(key) if key is not None else None, nk)
    if rc:
        raise _err("Unable to get next key", rc)
    return nk.raw


def LookupBatch(fd, cursor, count, keySize, valueSize):
    """gf_map_lookup_batch (chunked dump): up to `count` entries after `cursor`
    (None = from the start).  Returns (keys uint8[n, keySize], values
    uint8[n, valueSize], next_cursor, done)."""
    keys = np.empty((count, keySize), np.uint8)
    vals = np.empty((count, valueSize), np.uint8)
    cin = C.c_uint64(cursor or 0)
    cout = C.c_uint64(0)
    n = C.c_uint32(count)
    rc = lib.gf_map_lookup_batch(fd, C.byref(cin) if cursor is not None else None, C.byref(cout),
                                 keys.ctypes.data, vals.ctypes.data, C.byref(n))
    if rc and rc != -errno.ENOENT:
        raise _err("Unable to dump map (batch)", rc)
    return keys[:n.value], vals[:n.value], cout.value, rc == -errno.ENOENT


def UpdateBatch(fd, keys, values, n, flags=BPF_ANY):
    done = C.c_uint32(0)
    rc = lib.gf_map_update_batch(fd, keys, values, n, flags, C.byref(done))
    if rc:
        raise _err(f"Unable to update element (batch, {done.value} applied)", rc)
    return done.value


def ObjPin(fd, pathname):
    """bpf.ObjPin, pkg/bpf/bpf.go:224-243."""
    rc = lib.gf_obj_pin(fd, pathname.encode())
    if rc:
        raise _err("Unable to pin object", rc)


def ObjGet(pathname):
    """bpf.ObjGet, pkg/bpf/bpf.go:246-266 (handle 0 is an error)."""
    rc = lib.gf_obj_get(pathname.encode())
    if rc <= 0:
        raise _err(f"Unable to get object {pathname}", rc if rc < 0 else -errno.ENOENT)
    return rc


def ObjClose(fd):
    """bpf.ObjClose, pkg/bpf/bpf.go:269-274."""
    if fd > 0:
        rc = lib.gf_obj_close(fd)
        if rc:
            raise _err("Unable to close object", rc)


class MapInfo:
    def __init__(self, i):
        self.MapType = i.map_type
        self.KeySize = i.key_size
        self.ValueSize = i.value_size
        self.MaxEntries = i.max_entries
        self.Flags = i.map_flags
        self.Entries = i.n_entries
        self.DeviceBytes = i.device_bytes
        self.XferD2H = i.xfer_d2h
        self.XferH2D = i.xfer_h2d


def GetMapInfo(fd):
    """bpf.GetMapInfo (pkg/bpf/map.go:171-209) without /proc/<pid>/fdinfo."""
    i = gf_map_info()
    rc = lib.gf_map_get_info(fd, C.byref(i))
    if rc:
        raise _err("Unable to get map info", rc)
    return MapInfo(i)


def OpenOrCreateMap(path, mapType, keySize, valueSize, maxEntries, flags=0):
    """bpf.OpenOrCreateMap, pkg/bpf/bpf.go:343-419: reuse a pinned map whose
    properties match (objCheck, :276-341), otherwise (re)create and pin it.
    Returns (fd, isNewMap)."""
    rc = lib.gf_obj_get(path.encode())
    if rc > 0:
        info = GetMapInfo(rc)
        if (info.MapType, info.KeySize, info.ValueSize, info.MaxEntries, info.Flags) == (
                mapType, keySize, valueSize, maxEntries, flags):
            return rc, False
        ObjClose(rc)
        lib.gf_obj_unpin(path.encode())   # os.Remove(path)
    fd = CreateMap(mapType, keySize, valueSize, maxEntries, flags)
    ObjPin(fd, path)
    return fd, True


def GetMtime():
    """bpf.GetMtime, pkg/bpf/bpf.go:426-435 (seconds granularity here)."""
    return lib.gf_now_sec() * 1000000000


class Map:
    """bpf.Map object layer, pkg/bpf/map.go:115-498 (byte keys/values)."""

    def __init__(self, name, mapType, keySize, valueSize, maxEntries, flags=0, path=None):
        self.name = name
        self.path = path or MapPath(name)
        self.MapType, self.KeySize, self.ValueSize = mapType, keySize, valueSize
        self.MaxEntries, self.Flags = maxEntries, flags
        self.fd = 0

    def OpenOrCreate(self):
        self.fd, new = OpenOrCreateMap(self.path, self.MapType, self.KeySize, self.ValueSize,
                                       self.MaxEntries, self.Flags)
        return new

    def GetFd(self):
        return self.fd

    def Close(self):
        if self.fd:
            ObjClose(self.fd)
            self.fd = 0

    def Lookup(self, key):
        return LookupElement(self.fd, key, self.ValueSize)

    def Update(self, key, value, flags=BPF_ANY):
        UpdateElement(self.fd, key, value, flags)

    def Delete(self, key):
        DeleteElement(self.fd, key)

    def GetNextKey(self, key):
        return GetNextKey(self.fd, key, self.KeySize)

    def DumpWithCallback(self, cb, chunk=4096):
        """map.go:319-369: cb(key, value) for every entry (chunked dump)."""
        cursor, done = None, False
        while not done:
            k, v, cursor, done = LookupBatch(self.fd, cursor, chunk, self.KeySize, self.ValueSize)
            for i in range(len(k)):
                cb(k[i].tobytes(), v[i].tobytes())

    def DumpArrays(self, chunk=1 << 20):
        """Every entry as (keys uint8[n, KeySize], values uint8[n, ValueSize])."""
        ks, vs = [], []
        cursor, done = None, False
        while not done:
            k, v, cursor, done = LookupBatch(self.fd, cursor, chunk, self.KeySize, self.ValueSize)
            ks.append(k); vs.append(v)
        return np.concatenate(ks), np.concatenate(vs)

    def DumpKeyByKey(self, cb):
        """The reference loop itself: GetNextKey + LookupElement per entry."""
        key = None
        while True:
            try:
                nk = GetNextKey(self.fd, key, self.KeySize)
            except BPFError as e:
                if e.errno == errno.ENOENT:
                    return
                raise
            try:
                v = LookupElement(self.fd, nk, self.ValueSize)
            except BPFError as e:
                if e.errno == errno.ENOENT:   # deleted under us
                    key = nk
                    continue
                raise
            cb(nk, v)
            key = nk

    def Dump(self):
        out = {}
        self.DumpWithCallback(lambda k, v: out.__setitem__(k, v))
        return out

    def DeleteAll(self):
        keys = []
        self.DumpWithCallback(lambda k, v: keys.append(k))
        for k in keys:
            self.Delete(k)
