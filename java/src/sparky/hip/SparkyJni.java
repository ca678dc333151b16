// Sparky-compatible driver over the JNI binding (JDK 8..21, the Spark 1.x era's JVMs): the same
// host logic as SparkyHip (SparkyHost), so on a JDK 8 the "(url,rank)" lines carry JDK 8's own
// Double.toString digits, byte for byte what Sparky.java:237 wrote there.  Java 8 syntax only.
//
//   java -Djava.library.path=<dir of libpagerank_jni.so> -cp java/build/sparky-hip-jni.jar \
//        sparky.hip.SparkyJni <edge-list> [iterations=10] [--out DIR] [--save-every-iter]
//        [--dangling=local|none] [--device N] [--quiet] [--resume DIR/PageRank<i>]
package sparky.hip;

public final class SparkyJni {
    private SparkyJni() {}

    public static void main(String[] args) throws Throwable {
        SparkyHost.main(args, new SparkyHost.Engine() {
            @Override
            public double[] run(int device, int nVertices, int[] src, int[] dst, int flags, int iterations,
                                double[] initRanks, IterationListener listener, boolean ranksInCallback) {
                return PageRankJni.run(device, nVertices, src, dst, flags, iterations, initRanks, listener,
                        ranksInCallback);
            }
        });
    }
}
