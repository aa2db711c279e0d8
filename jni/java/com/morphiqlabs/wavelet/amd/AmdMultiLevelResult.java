package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.modwt.MultiLevelMODWTResult;

/**
 * A decomposition computed by the engine, as core/modwt/MultiLevelMODWTResultImpl.java: defensive copies
 * from the getters, energies summed sequentially in index order (computeEnergy, :211-216) and the total
 * as approximation first then levels 1..J (:109-117), level checks with the reference's message.
 */
final class AmdMultiLevelResult implements MultiLevelMODWTResult {
    private final double[][] details;  // [levels][n], level 1 first
    private final double[] approx;
    private Double totalEnergy;
    private double[] relative;

    AmdMultiLevelResult(double[][] details, double[] approx) {
        this.details = details;
        this.approx = approx;
    }

    @Override
    public int getLevels() {
        return details.length;
    }

    @Override
    public int getSignalLength() {
        return approx.length;
    }

    @Override
    public double[] getDetailCoeffsAtLevel(int level) {
        check(level);
        return details[level - 1].clone();
    }

    @Override
    public double[] getApproximationCoeffs() {
        return approx.clone();
    }

    @Override
    public double getDetailEnergyAtLevel(int level) {
        check(level);
        return energy(details[level - 1]);
    }

    @Override
    public double getApproximationEnergy() {
        return energy(approx);
    }

    @Override
    public double getTotalEnergy() {
        if (totalEnergy == null) {
            double t = getApproximationEnergy();
            for (int l = 1; l <= details.length; l++) t += getDetailEnergyAtLevel(l);
            totalEnergy = t;
        }
        return totalEnergy;
    }

    @Override
    public double[] getRelativeEnergyDistribution() {
        if (relative == null) {
            final double total = getTotalEnergy();
            relative = new double[details.length + 1];
            if (total != 0.0) {
                relative[0] = getApproximationEnergy() / total;
                for (int l = 1; l <= details.length; l++) relative[l] = getDetailEnergyAtLevel(l) / total;
            }
        }
        return relative.clone();
    }

    @Override
    public MultiLevelMODWTResult copy() {
        double[][] d = new double[details.length][];
        for (int l = 0; l < details.length; l++) d[l] = details[l].clone();
        return new AmdMultiLevelResult(d, approx.clone());
    }

    @Override
    public boolean isValid() {
        if (!finite(approx)) return false;
        for (double[] d : details) {
            if (d == null || d.length != approx.length || !finite(d)) return false;
        }
        return true;
    }

    private void check(int level) {
        if (level < 1 || level > details.length) {
            throw new IllegalArgumentException("Level " + level + " out of range [1, " + details.length + "]");
        }
    }

    private static double energy(double[] c) {
        double e = 0.0;
        for (double v : c) e += v * v;
        return e;
    }

    private static boolean finite(double[] c) {
        for (double v : c) {
            if (!Double.isFinite(v)) return false;
        }
        return true;
    }
}
