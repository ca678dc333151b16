// Sparky-compatible driver over the Panama FFM binding (JDK 22+): the process-level drop-in for
// the Spark job with the host logic in the reference's own language (SparkyHost; the JNI driver
// SparkyJni runs the same logic on JDK 8..21).
//
//   java --enable-native-access=ALL-UNNAMED -cp java/build/sparky-hip.jar sparky.hip.SparkyHip \
//        <edge-list> [iterations=10] [--out DIR] [--save-every-iter] [--dangling=local|none]
//        [--device N] [--quiet] [--resume DIR/PageRank<i>]
package sparky.hip;

public final class SparkyHip {
    private SparkyHip() {}

    public static void main(String[] args) throws Throwable {
        SparkyHost.main(args, (device, nVertices, src, dst, flags, iterations, initRanks, listener, ranksInCb) -> {
            try (PageRankHip g = new PageRankHip(device, nVertices, src, dst, flags)) {
                return g.run(iterations, initRanks, listener, ranksInCb);
            }
        });
    }
}
