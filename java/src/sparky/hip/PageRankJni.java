// JNI binding of libpagerank_hip for JDKs without the final FFM API (8..21): the same run as
// PageRankHip.run through java/jni/pagerank_jni.c (libpagerank_jni.so, linked against
// libpagerank_hip.so).  Non-zero status -> RuntimeException(pr_last_error()).  Java 8 syntax; no
// java.lang.foreign anywhere on this path (tests/test_java_host.py checks it).
package sparky.hip;

public final class PageRankJni {
    /** PR_ABI_VERSION of include/pagerank_hip.h this binding was written against. */
    public static final int ABI_VERSION = 2;
    public static final int PR_DANGLING_LOCAL = 0, PR_DANGLING_NONE = 1;

    static {
        System.loadLibrary("pagerank_jni");
        int v = abiVersion();
        if (v != ABI_VERSION)
            throw new UnsatisfiedLinkError("libpagerank_hip ABI " + v + ", this binding needs " + ABI_VERSION);
    }

    private PageRankJni() {}

    /** pr_abi_version() of the loaded libpagerank_hip. */
    public static native int abiVersion();

    /** Sparky.java:124-238 in one call: build (flags: 0 local / 1 none), then iterations; listener may be null. */
    public static native double[] run(int device, int nVertices, int[] src, int[] dst, int flags, int iterations,
                                      double[] initRanks, IterationListener listener, boolean ranksInCallback);
}
