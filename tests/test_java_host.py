"""The Java host of the drop-in (java/): Panama FFM binding, Sparky-compatible driver, JNI glue.

No JDK exists in this image, so on CPU the checks are structural: every symbol the FFM binding
looks up is declared by include/pagerank_hip.h with the arity of its FunctionDescriptor, and the
JNI glue compiles (gcc -fsyntax-only) against a minimal jni.h declaring only what it uses.  Where
javac exists, the sources are compiled too."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

JAVA = os.path.join(ROOT, "java")


def c_prototypes():
    hdr = open(os.path.join(ROOT, "include", "pagerank_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(pr_[a-z_]+)\s*\(([^;{]*?)\)\s*;", hdr, flags=re.S):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return protos


def test_ffm_binding_matches_the_c_abi():
    src = open(os.path.join(JAVA, "src", "sparky", "hip", "PageRankHip.java")).read()
    protos = c_prototypes()
    bound = re.findall(r'h\("(pr_[a-z_]+)", FunctionDescriptor\.(of|ofVoid)\(([^;]*?)\)\);', src, flags=re.S)
    assert {b[0] for b in bound} >= {"pr_graph_create", "pr_run", "pr_graph_info", "pr_graph_destroy", "pr_last_error"}
    for name, kind, args in bound:
        assert name in protos, name
        layouts = [a.strip() for a in args.split(",") if a.strip()]
        n_params = len(layouts) - (1 if kind == "of" else 0)  # of(ret, params...)
        assert n_params == protos[name], (name, n_params, protos[name])
    # the upcall descriptor mirrors pr_iter_cb (int32, const double*, 3 x double, void*)
    assert "FunctionDescriptor.ofVoid(\n            JAVA_INT, ADDRESS, JAVA_DOUBLE, JAVA_DOUBLE, JAVA_DOUBLE, ADDRESS)" in src
    # flag constants equal the header's
    hdr = open(os.path.join(ROOT, "include", "pagerank_hip.h")).read()
    for name in ("PR_DANGLING_NONE", "PR_NO_CANONICAL", "PR_CB_RANKS", "PR_INFO_COUNT"):
        v = int(re.search(rf"#define {name} \(?(\d+)u?\)?", hdr).group(1))
        assert re.search(rf"\b{name} = {v}\b", src), name


def java_sources():
    d = os.path.join(JAVA, "src", "sparky", "hip")
    return {f[:-5]: open(os.path.join(d, f)).read() for f in os.listdir(d) if f.endswith(".java")}


def jni_closure(srcs):
    """Classes of this package the JNI driver reaches (through any reference in their text)."""
    seen, todo = set(), ["SparkyJni", "PageRankJni"]
    while todo:
        c = todo.pop()
        if c in seen:
            continue
        seen.add(c)
        body = re.sub(r"//[^\n]*|/\*.*?\*/", "", srcs[c], flags=re.S)  # comments may name anything
        todo += [o for o in srcs if o != c and re.search(rf"\b{o}\b", body)]
    return seen


def test_jni_path_has_no_ffm_and_java8_syntax():
    """the JNI path must compile on JDK 8..21 -- no java.lang.foreign in any class it
    reaches, directly or through a referenced class, and no post-Java-8 syntax or API."""
    srcs = java_sources()
    closure = jni_closure(srcs)
    assert closure == {"SparkyJni", "PageRankJni", "SparkyHost", "IterationListener"}, closure
    java9plus = [r"\.strip\(\)", r"\bPath\.of\(", r"\bList\.of\(", r"\bMap\.of\(", r"\bSet\.of\(",
                 r"\bvar\s+\w+\s*=", r"case [^:\n]*->", r"\.isBlank\(\)", r'\"\"\"', r"\brecord\s+\w+\s*\(",
                 r"Files\.readString", r"\.repeat\(", r"\btry\s*\(\s*\w+\s*\)"]
    for c in closure:
        body = re.sub(r"//[^\n]*|/\*.*?\*/", "", srcs[c], flags=re.S)
        assert "java.lang.foreign" not in body, c
        for pat in java9plus:
            assert not re.search(pat, body), (c, pat)
    # the FFM classes are outside the closure and are the only ones importing java.lang.foreign
    code = {c: re.sub(r"//[^\n]*|/\*.*?\*/", "", b, flags=re.S) for c, b in srcs.items()}
    assert [c for c in code if "java.lang.foreign" in code[c]] == ["PageRankHip"]


def test_bindings_check_the_abi_version():
    hdr = open(os.path.join(ROOT, "include", "pagerank_hip.h")).read()
    v = int(re.search(r"#define PR_ABI_VERSION (\d+)", hdr).group(1))
    srcs = java_sources()
    for c in ("PageRankJni", "PageRankHip"):
        assert re.search(rf"ABI_VERSION = {v};", srcs[c]), c
    glue = open(os.path.join(JAVA, "jni", "pagerank_jni.c")).read()
    for m in re.findall(r"public static native \w+(?:\[\])? (\w+)\(", srcs["PageRankJni"]):
        assert f"Java_sparky_hip_PageRankJni_{m}(" in glue, m


STUB_JNI = r"""
typedef int jint; typedef long long jlong; typedef unsigned char jboolean; typedef double jdouble; typedef int jsize;
typedef void *jobject; typedef jobject jclass, jintArray, jdoubleArray, jarray, jthrowable; typedef struct _jm *jmethodID;
#define JNIEXPORT
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
  jsize (*GetArrayLength)(JNIEnv *, jarray);
  jint *(*GetIntArrayElements)(JNIEnv *, jintArray, jboolean *);
  void (*ReleaseIntArrayElements)(JNIEnv *, jintArray, jint *, jint);
  jdouble *(*GetDoubleArrayElements)(JNIEnv *, jdoubleArray, jboolean *);
  void (*ReleaseDoubleArrayElements)(JNIEnv *, jdoubleArray, jdouble *, jint);
  jdoubleArray (*NewDoubleArray)(JNIEnv *, jsize);
  void (*SetDoubleArrayRegion)(JNIEnv *, jdoubleArray, jsize, jsize, const jdouble *);
  void (*CallVoidMethod)(JNIEnv *, jobject, jmethodID, ...);
  jboolean (*ExceptionCheck)(JNIEnv *);
  void (*DeleteLocalRef)(JNIEnv *, jobject);
  jclass (*FindClass)(JNIEnv *, const char *);
  jint (*ThrowNew)(JNIEnv *, jclass, const char *);
  jclass (*GetObjectClass)(JNIEnv *, jobject);
  jmethodID (*GetMethodID)(JNIEnv *, jclass, const char *, const char *);
};
"""


def test_jni_glue_compiles(tmp_path):
    (tmp_path / "jni.h").write_text(STUB_JNI)
    res = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", f"-I{tmp_path}", f"-I{ROOT}/include",
                          os.path.join(JAVA, "jni", "pagerank_jni.c")], capture_output=True, text=True)
    assert res.returncode == 0, res.stderr


def test_javac_when_available(tmp_path):
    javac = shutil.which("javac")
    if not javac:
        pytest.skip("no JDK in this image: the Java host is compiled only where javac exists")
    srcs = [os.path.join(JAVA, "src", "sparky", "hip", f) for f in os.listdir(os.path.join(JAVA, "src", "sparky", "hip"))]
    d = os.path.join(JAVA, "src", "sparky", "hip")
    jni = [os.path.join(d, f + ".java") for f in ("IterationListener", "PageRankJni", "SparkyHost", "SparkyJni")]
    res = subprocess.run([javac, "--release", "8", "-d", str(tmp_path / "jni")] + jni, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr
    res = subprocess.run([javac, "--release", "22", "-d", str(tmp_path)] + srcs, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr
