// JNI binding of libpagerank_hip for JDKs without the final FFM API (8..21): the same run as
// PageRankHip.run through java/jni/pagerank_jni.c (libpagerank_jni.so, linked against
// libpagerank_hip.so).  Non-zero status -> RuntimeException(pr_last_error()).
package sparky.hip;

public final class PageRankJni {
    static {
        System.loadLibrary("pagerank_jni");
    }

    private PageRankJni() {}

    /** Sparky.java:124-238 in one call: build (flags: 0 local / 1 none), then iterations; listener may be null. */
    public static native double[] run(int device, int nVertices, int[] src, int[] dst, int flags, int iterations,
                                      double[] initRanks, PageRankHip.IterationListener listener,
                                      boolean ranksInCallback);
}
